"""GPU tests of the alternative LLR sources (direct / hard-reverse reconciliation)
and of the batched Monte-Carlo driver against the reference's outputs and the oracle."""
import ctypes as C

import numpy as np
import pytest

from conftest import assert_bit_exact, assert_llr_close, golden

import oracle as O

pytestmark = pytest.mark.gpu

KEYS = [("b1_s20", 1), ("b2_s30", 2), ("b2_s95", 2), ("b4_s130", 4), ("b4_s250", 4)]


def _col(arr, ld=64, dtype=None):
    """One frame in column 0 of a frame-innermost [n, ld] device tensor."""
    import torch

    a = np.asarray(arr)
    t = torch.zeros((a.size, ld), dtype=dtype or torch.float64, device="cuda")
    t[:, 0] = torch.from_numpy(a.copy())
    return t


@pytest.mark.parametrize("key,bps", KEYS)
def test_direct_and_bare_llr_vs_reference(gpu, key, bps):
    import torch
    import qamr
    from qamr import _lib

    g = golden("llr_sources.npz")
    two_var = float(g[f"{key}_two_var"])
    pa = qamr.PAMAlphabet(bps, 2.0)
    nm = qamr.NoiseMapper(pa, two_var / 2)
    y = g[f"{key}_y"]
    S = y.size
    out = torch.empty((S * bps, 64), dtype=torch.float64, device="cuda")
    yt = _col(y)
    _lib.check(_lib.load().qr_direct_lappr_device(nm.handle, two_var, 1, 64, S, C.c_void_p(yt.data_ptr()),
                                                  C.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    assert_bit_exact(out[:, 0].cpu().numpy(), g[f"{key}_direct"])
    # bare-LLR table lookup: bit-exact (host table is bit-exact, lookup is a copy)
    x = g[f"{key}_x"]
    xt = _col(x, dtype=torch.int64)
    table = torch.tensor(nm.bare_llr_table, dtype=torch.float64, device="cuda")
    _lib.check(_lib.load().qr_bare_llr_device(bps, C.c_void_p(table.data_ptr()), 1, 64, S, C.c_void_p(xt.data_ptr()),
                                              C.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    assert np.array_equal(out[:, 0].cpu().numpy(), g[f"{key}_base_bare_llr_x"])


@pytest.mark.parametrize("mode", ["softening", "direct", "hard"])
def test_simulator_batch_vs_oracle(gpu, mode):
    """One batch through Simulator.frames + decode + count; every frame re-decoded
    by the oracle and counted with utils.count_errors_from_lappr semantics."""
    import torch
    import qamr
    from qamr import codes
    from qamr.noisemapper import NoiseMapper
    from qamr.sim import Simulator

    vid, cid = codes.regular_code(1008)
    dec = qamr.Decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    sim = Simulator(dec, 2, mode, max_iterations=30, batch=96)
    snr = 3.5
    Es = sim.pa.variance
    nm = NoiseMapper(sim.pa, Es * (10 ** (-snr / 10)) / 2, sim.cfg if mode == "softening" else None)
    gen = torch.Generator(device="cuda").manual_seed(5)
    lappr, synd, word, ld = sim.frames(nm, 96, gen, Es * (10 ** (-snr / 10)))
    fin, succ, its = dec.decode_device(lappr, synd, 96, 30)
    torch.cuda.synchronize()
    L = lappr[:, :96].cpu().numpy().T.copy()
    Sy = synd[:, :96].cpu().numpy().T.copy()
    W = word[:, :96].cpu().numpy().T.copy()
    for f in range(0, 96, 7):
        assert np.array_equal(Sy[f], orc.eval_syndrome(W[f]))
    s2, i2, f2 = orc.decode_batch(L, Sy, 30)
    assert np.array_equal(succ.cpu().numpy(), s2) and np.array_equal(its.cpu().numpy(), i2)
    F1 = fin[:, :96].cpu().numpy().T
    assert_bit_exact(F1, f2)


def test_run_snr_and_cli(gpu, tmp_path):
    import qamr
    from qamr import codes
    from qamr.sim import Simulator
    from qamr.sim_reconciliation import main

    vid, cid = codes.regular_code(1008)
    dec = qamr.Decoder(vid, cid)
    for mode in ("softening", "direct", "hard"):
        snr, ber, fer, it = Simulator(dec, 2, mode, 20, batch=128).run_snr(2.0, 300, 10, seed=1)
        assert snr == 2.0 and 0 <= ber <= 1 and 0 <= fer <= 1 and it >= 0
    # early stop: many frame errors at low SNR -> stops after > loops/20 frames, at batch granularity
    snr, ber, fer, it = Simulator(dec, 2, "softening", 5, batch=64).run_snr(-5.0, 10000, 1, seed=2)
    assert fer == 1.0
    p = tmp_path / "code.csv"
    codes.save_edge_csv(str(p), vid, cid)
    out = tmp_path / "out.csv"
    rows = main([str(p), "--out", str(out), "--snr", "3", "8", "--nsnr", "2", "--simloops", "256",
                 "--batch", "128", "--maxiter", "30"])
    assert len(rows) == 2 and rows[1][2] <= rows[0][2]  # FER decreases with SNR
    lines = open(out).read().splitlines()
    assert lines[0] == ",EsN0dB,ber,fer,iters" and len(lines) == 3


def _reference_loop(frames, K, simulation_loops, ferr_count_min):
    """sims/reconciliation.pyx:127-168 verbatim over per-frame (success, iterations, final,
    word) in frame order: the counters and the stop at the first frame where the rule holds."""
    err_count = frame_error_count = decoding_iterations = successful_decoding = 0
    wordcount = -1
    for wordcount in range(simulation_loops):
        success, iterations, final, word = frames[wordcount]
        if success:
            decoding_iterations += iterations
            successful_decoding += 1
        new_errors = O.count_errors_from_lappr(final[:K], word[:K])
        if new_errors:
            frame_error_count += 1
            err_count += new_errors
        if frame_error_count >= ferr_count_min and wordcount > simulation_loops / 20:
            break
    wordcount += 1
    return (err_count / (wordcount * K), frame_error_count / wordcount,
            0 if successful_decoding == 0 else decoding_iterations / successful_decoding), wordcount


@pytest.mark.parametrize("loops,ferr_min,batch,snr", [(400, 7, 64, 1.8), (300, 40, 48, 2.2), (120, 1000, 64, 1.8)])
def test_run_snr_exact_early_stop(gpu, loops, ferr_min, batch, snr):
    """Simulator.run_snr stops at the reference's frame, not at a batch boundary: the GPU's own
    frames (captured through the hook) re-decoded one by one by the oracle and run through the
    reference's sequential loop give the same (snr, ber, fer, iters) tuple."""
    import torch
    import qamr
    from qamr import codes
    from qamr.sim import Simulator

    vid, cid = codes.regular_code(1008)
    dec = qamr.Decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    sim = Simulator(dec, 2, "softening", max_iterations=30, batch=batch)
    seen = []

    def hook(bidx, lappr, synd, word, B):
        torch.cuda.synchronize()
        seen.append((bidx, lappr[:, :B].cpu().numpy().T.copy(), synd[:, :B].cpu().numpy().T.copy(),
                     word[:, :B].cpu().numpy().T.copy()))

    got = sim.run_snr(snr, loops, ferr_min, seed=4, hook=hook)
    frames = []
    for bidx, L, Sy, W in sorted(seen, key=lambda t: t[0]):
        s, i, f = orc.decode_batch(L, Sy, 30)
        frames += [(int(s[k]), int(i[k]), f[k], W[k]) for k in range(L.shape[0])]
    ref, stop = _reference_loop(frames, sim.K, loops, ferr_min)
    assert got == (snr,) + ref, (got, ref, stop)
    if ferr_min < 1000:
        assert stop < loops and stop % batch != 0, stop   # the stop fell inside a batch
    else:
        assert stop == loops
