"""The exact schedule bench.py times, checked against the oracle and the reference.

bench.py decodes B = 4096 frames (ld = 4096) with the default tuning: the two-stream
split schedule (``split = 3``: check sweeps of one frame half on the caller's stream
beside the variable sweeps of the other half on a second stream) and active-frame
compaction (``compact = 1``).  The N=64800 bit-exact tests elsewhere run B = 24
(ld = 64), which takes ``run_flat``; here the batches are large enough (ld >= 512) that
``decode_batch_device`` takes ``run_split2`` with compaction, as in the timed region.

* ``test_timed_schedule_vs_oracle``: configs[2] (4-PAM 3.0 dB, B = 4096 = the bench's
  own batch), 4-PAM 3.6 dB (both outcomes occur, so compaction reshuffles lanes), and
  configs[3] (16-PAM 13.0 dB, demap fused, B = 4096): 16 frames spread over both halves
  decoded by the oracle from the GPU's LAPPRs -- success, iterations and final LAPPRs
  bit-exact; for 16-PAM the GPU-demapped LAPPRs of those frames too
  (reference: decoder.pyx:424-433, noisemapper.pyx:544-559).
* ``test_reference_frames_in_timed_batch``: the frames the reference itself demapped
  and decoded (tests/golden/dvbs2.npz, dvbs2_16pam.npz) planted into such batches at a
  column of each half: demapped LAPPRs, success, iterations and final LAPPRs identical
  to the reference's (sims/reconciliation.pyx:143-147).
"""
import numpy as np
import pytest

from conftest import assert_bit_exact, golden

import oracle as O

pytestmark = pytest.mark.gpu

# the tuning bench.py runs with (csrc/decoder.hip Tuning defaults)
TIMED = dict(split=3, compact=1)


def _assert_timed_defaults():
    from qamr import _lib
    for k, v in TIMED.items():
        assert int(_lib.tune_get(k)) == v, f"bench default {k}={v} changed: update this test"


def _pipeline(bps, snr, B, seed, max_iterations=50):
    import torch
    import qamr
    from qamr import codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.dvbs2_like_half()
    dec = qamr.Decoder(vid, cid)
    pipe = SofteningPipeline(dec, bps=bps, snr_db=snr, batch=B, max_iterations=max_iterations)
    assert pipe.ld % 512 == 0 and B > pipe.ld - 256  # run_split2 territory
    b = pipe.generate(torch.Generator(device="cuda").manual_seed(seed))
    return vid, cid, dec, pipe, b


def _cols(B, n=16):
    """n frame columns spread over both halves of the split schedule."""
    return np.unique(np.r_[np.linspace(0, B // 2 - 1, n // 2).astype(int),
                           np.linspace(B // 2, B - 1, n // 2).astype(int)])


@pytest.mark.parametrize("bps,snr,B", [(2, 3.0, 4096), (2, 3.6, 512), (4, 13.0, 4096)])
def test_timed_schedule_vs_oracle(gpu, bps, snr, B):
    import torch

    _assert_timed_defaults()
    vid, cid, dec, pipe, b = _pipeline(bps, snr, B, seed=100 + int(10 * snr))
    lappr = pipe.demap(b)
    fin, succ, its = pipe.decode(lappr, b)
    torch.cuda.synchronize()
    cols = _cols(B)
    ct = torch.as_tensor(cols, device=lappr.device)
    L = lappr[:, ct].T.contiguous().cpu().numpy()
    Sy = b.synd[:, ct].T.contiguous().cpu().numpy()
    if bps == 4:
        onm = O.OracleNoiseMapper(bps, 2.0, pipe.noise_var, np.array([0, 1] * 8, np.uint8))
        nh = b.nhat[:, ct].T.contiguous().cpu().numpy()
        xs = b.x[:, ct].T.contiguous().cpu().numpy()
        ref_l = np.stack([onm.demap_lappr_array(nh[i], xs[i]) for i in range(len(cols))])
        assert_bit_exact(L, ref_l)
    s2, i2, f2 = O.OracleCode(vid, cid).decode_batch(L, Sy, 50)
    assert np.array_equal(succ[ct].cpu().numpy(), s2)
    assert np.array_equal(its[ct].cpu().numpy(), i2)
    assert_bit_exact(fin[:, ct].T.contiguous().cpu().numpy(), f2)
    if snr == 3.6:
        s_all = succ.cpu().numpy()
        assert 0 < s_all.sum() < B  # frames stop at different iterations: compaction is exercised


@pytest.mark.parametrize("fname,key,bps,snr,B", [("dvbs2.npz", "snr30", 2, 3.0, 4096),
                                                 ("dvbs2.npz", "snr40", 2, 4.0, 512),
                                                 ("dvbs2_16pam.npz", "snr130", 4, 13.0, 4096),
                                                 ("dvbs2_16pam.npz", "snr145", 4, 14.5, 512)])
def test_reference_frames_in_timed_batch(gpu, fname, key, bps, snr, B):
    import torch
    from qamr import codes

    _assert_timed_defaults()
    g = golden(fname)
    vid, cid, dec, pipe, b = _pipeline(bps, snr, B, seed=7)
    assert codes.code_digest(vid, cid) == str(g["digest"])
    assert pipe.noise_var == float(g[f"{key}_noise_var"])
    dev = b.x.device
    x = torch.as_tensor(g[f"{key}_x"].astype(np.int64), device=dev)
    nh = torch.as_tensor(g[f"{key}_nhat"], device=dev)
    sy = torch.as_tensor(np.unpackbits(g[f"{key}_synd_packed"])[:dec.cnum], device=dev)
    plant = [B // 2 - 37, B - 5]  # one column in each half
    for c in plant:
        b.x[:, c] = x
        b.nhat[:, c] = nh
        b.synd[:, c] = sy
    lappr = pipe.demap(b)
    fin, succ, its = pipe.decode(lappr, b)
    torch.cuda.synchronize()
    for c in plant:
        assert_bit_exact(lappr[:, c].cpu().numpy(), g[f"{key}_lappr"])
        assert (int(succ[c]), int(its[c])) == (int(g[f"{key}_success"]), int(g[f"{key}_iters"]))
        f = fin[:, c].cpu().numpy()
        assert np.array_equal(np.packbits(f < 0), g[f"{key}_hard_packed"])
        if f"{key}_final" in g:
            assert_bit_exact(f, g[f"{key}_final"])
        else:
            assert_bit_exact(f[g[f"{key}_sample_idx"]], g[f"{key}_sample_final"])


@pytest.mark.parametrize("bps,snr,B,mi", [(2, 4.0, 4096, 50), (4, 14.5, 4096, 50), (2, 4.0, 1024, 50),
                                          (4, 14.5, 1024, 50), (2, 3.8, 2048, 50), (2, 4.0, 1000, 50),
                                          (2, 4.0, 1024, 22)])
def test_column_repack_vs_oracle(gpu, bps, snr, B, mi):
    """Converging batches under the column repack (knob repack, default on: when a range's
    running frames fill at most knob repack_pct percent of its columns, the device gathers them
    into the front columns of the work set's other column set), incl. the bench's own B = 4096
    batches of its converging operating points (BENCH op_dvbs2_4pam_4.0dB /
    op_dvbs2_16pam_14.5dB): every frame identical to the run with no repack at all, the frames
    that ran longest -- the ones that went through the repacks -- and frames spread over both
    ranges bit-exact against the oracle, and the device did repack.  Each repack's first variable
    and check sweeps read the messages at the frames' old columns of the old set (the transition:
    k_repack_rows moves no message).  On the bench's 4-PAM 4.0 dB batch a range repacks more than
    once (column set 1 -> 0 as well as 0 -> 1) and ends at most 64 columns wide, so its last
    iterations ran the narrow sweeps (lanes = node x frame, check_narrow / var_narrow_sweep)
    (reference: decoder.pyx:424-436)."""
    import torch
    from qamr import _lib

    _assert_timed_defaults()
    vid, cid, dec, pipe, b = _pipeline(bps, snr, B, seed=300 + int(10 * snr), max_iterations=mi)
    lappr = pipe.demap(b)
    # the default (repack_pct 80: repacks early and often, transitions at consecutive decision
    # points; row-move grid 128); no repack; an odd 7-workgroup grid (each walks many row groups);
    # repacks at 50 % with a 1 024-workgroup grid
    runs = [dict(), dict(repack=0), dict(repack_grid=7), dict(repack_pct=50, repack_grid=1024)]
    names = ("repack", "repack_pct", "repack_grid")
    saved = {k: _lib.tune_get(k) for k in names}
    outs, stats = [], []
    try:
        for t in runs:
            for k, v in saved.items():
                _lib.tune_set(k, t.get(k, v))
            outs.append([x.clone() for x in pipe.decode(lappr, b)])
            torch.cuda.synchronize()
            stats.append(dec.repack_stats(pipe.ld, mi))
    finally:
        for k, v in saved.items():
            _lib.tune_set(k, v)
    # the device repacked (no repack is decided before the last variable sweep: its transition
    # would end in the final parity sweep; with max_iterations 22 a 50 % threshold is first met there)
    (rep0, rep1), (w0, w1) = stats[0]
    assert rep0 + rep1 > 0, stats
    assert min(w0, w1) < pipe.ld // 2, stats
    assert stats[1] == ((0, 0), (pipe.ld // 2, pipe.ld // 2))  # repack off: never
    if (bps, snr, B) == (2, 4.0, 4096):
        assert max(rep0, rep1) >= 2, stats[0]  # both directions between the column sets
        assert min(w0, w1) <= 64, stats[0]     # the narrow sweeps ran
    f1, s1, i1 = outs[0]
    for f0, s0, i0 in outs[1:]:
        assert torch.equal(s1, s0) and torch.equal(i1, i0)
        assert torch.equal(f1[:, :B].view(torch.int64), f0[:, :B].view(torch.int64))
    its = i1.cpu().numpy()
    # the bench's own 4.0 dB batch: 64 frames more against the oracle, spread over both ranges
    # (every column set and transition a frame can go through before it stops)
    nspread = 72 if (bps, snr, B) == (2, 4.0, 4096) else 8
    cols = np.unique(np.r_[np.argsort(-its, kind="stable")[:8], _cols(B, nspread)])
    ct = torch.as_tensor(cols, device=lappr.device)
    L = lappr[:, ct].T.contiguous().cpu().numpy()
    Sy = b.synd[:, ct].T.contiguous().cpu().numpy()
    s2, i2, fo = O.OracleCode(vid, cid).decode_batch(L, Sy, mi)
    assert np.array_equal(s1[ct].cpu().numpy(), s2) and np.array_equal(i1[ct].cpu().numpy(), i2)
    assert_bit_exact(f1[:, ct].T.contiguous().cpu().numpy(), fo)


def test_repack_decode_is_asynchronous_and_capturable(gpu):
    """qr_decode_batch_device keeps its contract with the column repack on (include/qamr.h):
    on the bench's 4-PAM 4.0 dB B = 4096 batch the call returns while the GPU is still
    decoding (the host never waits: every repack decision is taken on the device), and a
    HIP-graph capture of the same decode replays bit-identically to the eager decode, the
    device repacking inside the graph."""
    import time

    import torch

    _assert_timed_defaults()
    B, mi = 4096, 50
    vid, cid, dec, pipe, b = _pipeline(2, 4.0, B, seed=340)
    lappr = pipe.demap(b)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        dec.decode_device(lappr, b.synd, B, mi)  # warm-up: allocates this stream's workspace
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        t0 = time.perf_counter()
        ref = dec.decode_device(lappr, b.synd, B, mi)
        t_ret = time.perf_counter() - t0
        end = torch.cuda.Event()
        end.record(s)
        pending = not end.query()
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    eager_stats = dec.repack_stats(pipe.ld, mi, stream=s)
    assert pending, (t_ret, t_all)
    assert sum(eager_stats[0]) > 0, eager_stats
    fin = torch.full_like(lappr, np.nan)
    succ = torch.zeros(B, dtype=torch.uint8, device=lappr.device)
    its = torch.zeros(B, dtype=torch.int32, device=lappr.device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        dec.decode_device(lappr, b.synd, B, mi, fin, succ, its)
    g.replay()
    torch.cuda.synchronize()
    graph_stats = dec.repack_stats(pipe.ld, mi, stream=s)
    assert sum(graph_stats[0]) > 0, graph_stats
    assert torch.equal(succ, ref[1]) and torch.equal(its, ref[2])
    assert torch.equal(fin[:, :B].view(torch.int64), ref[0][:, :B].view(torch.int64))


def test_repack_stats_after_resident_decode(gpu):
    """qr_decode_repack_stats reports "never repacked" (0 repacks, widths ld / 2) for a decode
    that took the frame-resident schedule (configs[1]'s reg-(3,6) N=1008), even on a workspace
    whose last two-stream decode did repack."""
    import torch
    import qamr
    from qamr import codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.regular_code(1008)
    dec = qamr.Decoder(vid, cid)
    pipe = SofteningPipeline(dec, bps=2, snr_db=3.0, batch=1024, max_iterations=20)
    b = pipe.generate(torch.Generator(device="cuda").manual_seed(5))
    lappr = pipe.demap(b)
    st = torch.cuda.current_stream()
    ws = dec._workspace(st, dec.workspace_bytes(pipe.ld, 20))
    ws.fill_(0x5A)  # garbage where the RangeSel block lives
    pipe.decode(lappr, b)
    torch.cuda.synchronize()
    assert dec.repack_stats(pipe.ld, 20) == ((0, 0), (pipe.ld // 2, pipe.ld // 2))
