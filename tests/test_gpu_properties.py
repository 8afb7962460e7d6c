"""Size-independent properties of the GPU decoder at the benchmark's full size, and
parity on graphs whose shape the goldens do not cover.

* irregular codes (check degrees 2..20, incl. the runtime-degree kernel above 16)
  against the oracle;
* the schedule and every tuning knob change nothing: split / flat schedule, check
  and variable geometries, non-temporal messages -> bit-identical outputs;
* a frame's result does not depend on the batch it is decoded in (permutation,
  sub-batch, repetition) at N=64800;
* at N=64800 the configs[2]/[3] operating points (4-PAM 3 dB, 16-PAM 13 dB: every
  frame runs 50 iterations without converging, the 16-PAM frames with LAPPRs in the
  hundreds, where a 1-ulp difference per box-plus grows past 1e-6) decode bit for bit
  like the oracle;
* at N=64800, B=4096 (BASELINE configs[2] size, 3.6 dB): every frame that
  reports success satisfies its syndrome with the returned hard decisions, every
  other frame ran max_iterations.
"""
import numpy as np
import pytest

from conftest import assert_bit_exact

import oracle as O

pytestmark = pytest.mark.gpu


def _decoder(vid, cid):
    import qamr
    return qamr.Decoder(np.asarray(vid, np.int64), np.asarray(cid, np.int64))


def _irregular_code(rng, C, degrees, V):
    """Checks with the given degree mix, sockets dealt at random over V variables
    (every variable used at least once)."""
    deg = rng.choice(degrees, C)
    E = int(deg.sum())
    sockets = np.concatenate([np.arange(V), rng.integers(0, V, E - V)])
    rng.shuffle(sockets)
    cid = np.repeat(np.arange(C), deg)
    return sockets.astype(np.int64), cid.astype(np.int64)


def test_irregular_degrees_vs_oracle(gpu):
    rng = np.random.default_rng(11)
    vid, cid = _irregular_code(rng, 120, [2, 3, 5, 7, 9, 16, 17, 20], 400)
    dec = _decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    B = 70
    word = rng.integers(0, 2, (B, 400)).astype(np.uint8)
    synd = np.stack([orc.eval_syndrome(w) for w in word])
    sig = rng.uniform(0.4, 0.9, B)[:, None]
    llr = 2 / sig ** 2 * ((1 - 2.0 * word) + sig * rng.standard_normal((B, 400)))
    s1, i1, f1 = dec.decode_batch(llr, synd, 40)
    s2, i2, f2 = orc.decode_batch(llr, synd, 40)
    assert np.array_equal(s1, s2) and np.array_equal(i1, i2)
    assert_bit_exact(f1, f2)


def _dvbs2_batch(B, snr_db, seed=0):
    import torch
    import qamr
    from qamr import codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.dvbs2_like_half()
    dec = qamr.Decoder(vid, cid)
    pipe = SofteningPipeline(dec, 2, snr_db, batch=B, max_iterations=50)
    batch = pipe.generate(torch.Generator(device="cuda").manual_seed(seed))
    lappr = pipe.demap(batch)
    return vid, cid, dec, pipe, batch, lappr


TUNINGS = [dict(split=1), dict(split=2, check_per=1), dict(check_ft=64, check_per=3, var_ft=128, var_per=1),
           dict(nt=0), dict(split=1, check_ft=128, var_per=16), dict(split=3, lds_pad_kb=0, nt=0),
           dict(split=2), dict(compact=0), dict(split=1, compact=0), dict(split=2, compact=0),
           dict(side=0, compact=0), dict(min_blocks=0), dict(min_blocks=4096, split=1),
           dict(split_min_blocks=4096), dict(split_min_blocks=0, min_blocks=0),
           dict(var_pace=0), dict(var_pace=3, var_per=1, compact=0), dict(var_pace=4096),
           dict(check_tail=0), dict(check_tail=3, check_per=7, compact=0), dict(check_tail=2, split=1),
           dict(var_boost=1), dict(var_boost=16, var_pace=3, var_per=1)]


def test_schedule_and_tuning_invariance(gpu):
    import torch
    from qamr import _lib

    _, _, dec, pipe, batch, lappr = _dvbs2_batch(320, 3.6, seed=1)
    names = ["split", "check_ft", "check_per", "var_ft", "var_per", "nt", "lds_pad_kb", "compact", "side", "min_blocks",
             "split_min_blocks", "var_pace", "check_tail", "var_boost"]
    saved = {k: _lib.tune_get(k) for k in names}
    try:
        ref = [x.clone() for x in dec.decode_device(lappr, batch.synd, batch.B, 50)]
        torch.cuda.synchronize()
        assert 0 < int(ref[1].sum()) < batch.B  # converging and failing frames
        for t in TUNINGS:
            for k, v in saved.items():
                _lib.tune_set(k, v)
            for k, v in t.items():
                _lib.tune_set(k, v)
            out = dec.decode_device(lappr, batch.synd, batch.B, 50)
            torch.cuda.synchronize()
            assert torch.equal(out[1], ref[1]) and torch.equal(out[2], ref[2]), t
            assert torch.equal(out[0][:, :batch.B].view(torch.int64), ref[0][:, :batch.B].view(torch.int64)), t
    finally:
        for k, v in saved.items():
            _lib.tune_set(k, v)


def test_batch_composition_invariance_full_size(gpu):
    import torch
    from qamr.pipeline import leading_dim

    _, _, dec, pipe, batch, lappr = _dvbs2_batch(256, 3.6, seed=2)
    B = batch.B
    f0, s0, i0 = [x.clone() for x in dec.decode_device(lappr, batch.synd, B, 50)]
    # repetition: deterministic
    f1, s1, i1 = dec.decode_device(lappr, batch.synd, B, 50)
    torch.cuda.synchronize()
    assert torch.equal(f0[:, :B].view(torch.int64), f1[:, :B].view(torch.int64))
    # permuted sub-batch of 77 frames in a fresh, differently padded buffer
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(3))[:77].to(lappr.device)
    ld = leading_dim(77)
    lp = torch.zeros((lappr.shape[0], ld), dtype=lappr.dtype, device=lappr.device)
    sp = torch.zeros((batch.synd.shape[0], ld), dtype=batch.synd.dtype, device=lappr.device)
    lp[:, :77] = lappr[:, perm]
    sp[:, :77] = batch.synd[:, perm]
    f2, s2, i2 = dec.decode_device(lp, sp, 77, 50)
    torch.cuda.synchronize()
    assert torch.equal(s2, s0[perm]) and torch.equal(i2, i0[perm])
    assert torch.equal(f2[:, :77].view(torch.int64), f0[:, perm].view(torch.int64))


def test_full_size_success_implies_syndrome(gpu):
    """BASELINE configs[2] size (N=64800, B=4096) at 3.6 dB (between the 3.0 dB worst
    case and the 4.0 dB operating point, so both outcomes occur): success <=> the
    returned hard decisions satisfy the syndrome (checked on the host for 512
    frames), failed frames ran all 50 iterations, iteration counts in [1, 50]."""
    import torch

    vid, cid, dec, pipe, batch, lappr = _dvbs2_batch(4096, 3.6, seed=4)
    fin, succ, its = dec.decode_device(lappr, batch.synd, batch.B, 50)
    torch.cuda.synchronize()
    s, it = succ.cpu().numpy(), its.cpu().numpy()
    assert 0 < s.sum() < 4096
    assert np.all(it[s == 0] == 50) and np.all((it[s == 1] >= 1) & (it[s == 1] <= 50))
    cols = np.arange(0, 4096, 8)
    hard = (fin[:, cols].cpu().numpy() < 0).astype(np.uint8)        # [V, 512]
    syn = batch.synd[:, cols].cpu().numpy()                          # [C, 512]
    order = np.argsort(cid, kind="stable")
    starts = np.flatnonzero(np.r_[True, np.diff(cid[order]) != 0])
    par = np.bitwise_xor.reduceat(hard[vid[order]], starts, axis=0)  # [C, 512]
    ok = ~np.any(par ^ syn, axis=0)
    assert np.array_equal(ok, s[cols] == 1)


@pytest.mark.parametrize("bps,snr", [(2, 3.0), (2, 4.0), (4, 13.0), (4, 14.5)])
def test_full_size_operating_points_bit_exact(gpu, bps, snr):
    """configs[2] / configs[3] frames (GPU-generated, GPU-demapped) decoded by libqamr
    and by the oracle from the same LAPPRs: identical bits after 50 iterations."""
    import torch
    import qamr
    from qamr import codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.dvbs2_like_half()
    dec = qamr.Decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    pipe = SofteningPipeline(dec, bps=bps, snr_db=snr, batch=24)
    gen = torch.Generator(device="cuda").manual_seed(77 + bps)
    b = pipe.generate(gen)
    lappr = pipe.demap(b)
    fin, succ, its = pipe.decode(lappr, b)
    torch.cuda.synchronize()
    L = lappr[:, :b.B].T.contiguous().cpu().numpy()
    Sy = b.synd[:, :b.B].T.contiguous().cpu().numpy()
    s2, i2, f2 = orc.decode_batch(L, Sy, 50)
    assert np.array_equal(succ.cpu().numpy(), s2) and np.array_equal(its.cpu().numpy(), i2)
    assert_bit_exact(fin[:, :b.B].T.contiguous().cpu().numpy(), f2)
