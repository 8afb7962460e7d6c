"""GPU parity tests of the soft demapper and the Bob-side producers against the
reference's golden outputs and the oracle.  The demapper's exp/log are glibc's,
restated bit for bit (glibc_math.hpp), and its erf is scipy's cephes erf: the
LAPPRs must equal the reference's bit for bit (conftest.assert_bit_exact)."""
import numpy as np
import pytest

from conftest import assert_bit_exact, assert_llr_close, golden

import oracle as O

pytestmark = pytest.mark.gpu

KEYS = [("b2_s30", 2), ("b2_s40", 2), ("b2_s95", 2), ("b4_s130", 4), ("b4_s145", 4), ("b4_s250", 4)]


def _nm(bps, nv, cfg=None):
    import qamr
    return qamr.NoiseMapper(qamr.PAMAlphabet(bps, 2.0), nv, cfg)


@pytest.mark.parametrize("key,bps", KEYS)
def test_tables_and_demap_vs_reference(gpu, key, bps):
    g = golden("demap.npz")
    nv = float(g[f"{key}_noise_var"])
    nm = _nm(bps, nv, g[f"{key}_cfg"])
    # host tables: scipy-exact erf in libqamr's host code -> bit-exact
    assert np.array_equal(nm.F_Y_thresholds, g[f"{key}_Fthr"])
    assert np.array_equal(nm.delta_F_Y, g[f"{key}_dF"])
    l = nm.demap_lappr_array(g[f"{key}_nhat"], g[f"{key}_x"])
    assert_bit_exact(l, g[f"{key}_lappr"])
    nm0 = _nm(bps, nv)
    assert_bit_exact(nm0.demap_lappr_array(g[f"{key}_nhat"][:20], g[f"{key}_x"][:20]), g[f"{key}_lappr_base"])


@pytest.mark.parametrize("key,bps", KEYS)
def test_bob_side_vs_reference(gpu, key, bps):
    g = golden("demap.npz")
    nm = _nm(bps, float(g[f"{key}_noise_var"]), g[f"{key}_cfg"])
    xh = nm.hard_decide_index(g[f"{key}_y"])
    assert np.array_equal(xh, g[f"{key}_xhat"])
    nh = nm.map_noise(g[f"{key}_y"], xh)
    assert_bit_exact(nh, g[f"{key}_nhat"])
    # the single-frame path lays the frame's symbols along the frame axis: Gray words too
    _, nh2, word = nm._bob_host(g[f"{key}_y"])
    assert_bit_exact(nh2, g[f"{key}_nhat"])
    assert np.array_equal(word, np.asarray(g[f"{key}_word"], np.uint8).ravel())


def test_single_frame_syndrome_vs_oracle(gpu):
    """Matrix.eval_syndrome (matrix.pyx:55-60) for one frame: lane = check node."""
    import qamr
    from qamr import codes
    from qamr.matrix import Matrix

    import oracle as O

    vid, cid = codes.regular_code(1008)
    mat = Matrix(vid, cid)
    orc = O.OracleCode(vid, cid)
    rng = np.random.default_rng(8)
    for _ in range(3):
        w = rng.integers(0, 2, 1008).astype(np.uint8)
        assert np.array_equal(mat.eval_syndrome(w), orc.eval_syndrome(w))


def test_demap_device_layout_and_alpha(gpu):
    """Batched demap writes the decoder's frame-innermost layout; alpha scales."""
    import torch

    g = golden("demap.npz")
    key, bps = "b2_s30", 2
    nm = _nm(bps, float(g[f"{key}_noise_var"]), g[f"{key}_cfg"])
    n, x = g[f"{key}_nhat"], g[f"{key}_x"]
    S = 100
    B, ld = 3, 64
    dev = torch.device("cuda", 0)
    nt = torch.zeros((S, ld), dtype=torch.float64, device=dev)
    xt = torch.zeros((S, ld), dtype=torch.int64, device=dev)
    for f in range(B):  # frame f = the golden symbols shifted by f
        nt[:, f] = torch.from_numpy(np.roll(n, f)[:S])
        xt[:, f] = torch.from_numpy(np.roll(x, f)[:S])
    out = nm.demap_device(nt, xt, B, alpha=0.75)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    ref = g[f"{key}_lappr"].reshape(-1, bps)
    for f in range(B):
        exp = (np.roll(ref, f, axis=0)[:S] * 0.75).reshape(-1)
        assert_bit_exact(o[:, f], exp)


def test_demap_random_vs_oracle(gpu):
    rng = np.random.default_rng(4)
    for bps, nv in ((1, 0.7), (2, 0.4), (3, 1.1), (4, 0.9)):
        M = 1 << bps
        cfg = rng.integers(0, 2, M).astype(np.uint8)
        nm = _nm(bps, nv, cfg)
        onm = O.OracleNoiseMapper(bps, 2.0, nv, cfg)
        S = 300
        n = rng.uniform(0, 1, S)
        n[:3] = [0.0, 1.0, 0.5]
        x = rng.integers(0, M, S)
        assert_bit_exact(nm.demap_lappr_array(n, x), onm.demap_lappr_array(n, x))


def test_demap_errors(gpu):
    nm = _nm(2, 1.0)
    with pytest.raises(ValueError):
        nm.demap_lappr_array(np.zeros(3), np.zeros(4, np.int64))
    with pytest.raises(ValueError):
        nm.demap_lappr_array(np.zeros(3, np.float32), np.zeros(3, np.int64))
    import qamr
    with pytest.raises(ValueError):
        qamr.NoiseMapper(qamr.PAMAlphabet(2, 2.0), 0.0)
    with pytest.raises(ValueError):
        qamr.NoiseMapper(qamr.PAMAlphabet(2, 2.0), 1.0, np.zeros(2, np.uint8))
    out = nm.demap_lappr_array(np.array([0.5]), np.array([7], np.int64))  # bad symbol index -> NaN
    assert np.isnan(out).all()


def test_syndrome_and_counters_vs_oracle(gpu):
    import torch
    import qamr
    from qamr import codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.regular_code(1008)
    dec = qamr.Decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    pipe = SofteningPipeline(dec, 2, 3.0, batch=130, max_iterations=20)
    gen = torch.Generator(device="cuda").manual_seed(1)
    b, l, fin, succ, its = pipe.run_batch(gen)
    torch.cuda.synchronize()
    word = b.word[:, :130].cpu().numpy().T.copy()
    synd = b.synd[:, :130].cpu().numpy().T
    for f in range(0, 130, 13):
        assert np.array_equal(synd[f], orc.eval_syndrome(word[f]))
    # Bob + demap vs oracle on a few frames
    onm = O.OracleNoiseMapper(2, 2.0, pipe.noise_var, np.array([0, 1, 0, 1], np.uint8))
    nh = b.nhat[:, :130].cpu().numpy().T
    xx = b.x[:, :130].cpu().numpy().T
    lap = l[:, :130].cpu().numpy().T
    for f in (0, 64, 129):
        assert_bit_exact(lap[f], onm.demap_lappr_array(nh[f], xx[f]))
    # decode vs oracle, then BER/FER counters vs utils.count_errors_from_lappr
    s2, i2, f2 = orc.decode_batch(lap, synd, 20)
    assert np.array_equal(succ.cpu().numpy(), s2) and np.array_equal(its.cpu().numpy(), i2)
    finv = fin[:, :130].cpu().numpy().T
    K = pipe.K
    errs = np.array([qamr.count_errors_from_lappr(finv[f, :K], word[f, :K]) for f in range(130)])
    c = pipe.counters.cpu().numpy()
    assert c[0] == errs.sum() and c[1] == (errs > 0).sum() and c[2] == s2.sum()
    assert c[3] == i2[s2 == 1].sum() and c[4] == 130


@pytest.mark.parametrize("bps,snr", [(1, 0.0), (2, 3.0), (2, 25.0), (3, 9.5), (4, 13.0), (4, 25.0), (4, 40.0)])
def test_fast_root_search_bit_identical_to_brute_force(gpu, bps, snr):
    """The Newton-located, replayed root search (default) returns the same doubles as
    the reference's brute-force bracket + bisection (qr_tune demap_fast=0) on every
    symbol: uniform n_hat, the edge values 0 / 1 / tiny, both sign configurations."""
    import torch
    from qamr import _lib

    pa = __import__("qamr").PAMAlphabet(bps, 2.0)
    nv = pa.variance * 10 ** (-snr / 10) / 2
    M = 1 << bps
    cfg = np.array([i & 1 for i in range(M)], np.uint8)
    nm = _nm(bps, nv, cfg)
    rng = np.random.default_rng(bps * 100 + int(snr))
    S, ld = 2000, 64
    n = rng.random((S, ld))
    n[0, :6] = [0.0, 1.0, 1e-300, 1e-17, 1 - 1e-16, 0.5]
    n[1:4] = rng.random((3, ld)) * 1e-12
    x = rng.integers(0, M, (S, ld))
    dev = torch.device("cuda", 0)
    nt = torch.from_numpy(n).to(dev).contiguous()
    xt = torch.from_numpy(x).to(dev).contiguous()
    try:
        _lib.tune_set("demap_fast", 1)
        fast = nm.demap_device(nt, xt, ld).clone()
        _lib.tune_set("demap_fast", 0)
        brute = nm.demap_device(nt, xt, ld).clone()
    finally:
        _lib.tune_set("demap_fast", 1)
    torch.cuda.synchronize()
    a, b = fast.cpu().numpy(), brute.cpu().numpy()
    same = (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), f"{(~same).sum()} LAPPRs differ"


@pytest.mark.parametrize("bps,snr", [(1, 2.0), (2, 3.0), (3, 9.5), (4, 13.0), (4, 25.0), (5, 20.0), (6, 30.0)])
def test_wave_private_demap_equals_per_symbol(gpu, bps, snr):
    """The wave-private demapper (default on 64-frame tiles: one wave walks all hypotheses of its
    tile, cooperative exact F_Y, Gray sums in i order in LDS) returns the per-symbol
    kernel's doubles bit for bit, on a ragged batch (B < ld) with out-of-range symbol
    indices (-> NaN) and both sign configurations; and its 2..16-PAM output matches the
    oracle (reference restatement) on sampled frames."""
    import torch
    from qamr import _lib

    pa = __import__("qamr").PAMAlphabet(bps, 2.0)
    nv = pa.variance * 10 ** (-snr / 10) / 2
    M = 1 << bps
    rng = np.random.default_rng(700 + bps)
    cfg = rng.integers(0, 2, M).astype(np.uint8)
    nm = _nm(bps, nv, cfg)
    S, ld, B = 257, 192, 131
    n = rng.random((S, ld))
    n[0, :5] = [0.0, 1.0, 1e-300, 1 - 1e-16, 0.5]
    x = rng.integers(0, M, (S, ld))
    x[1, :3] = [-1, M, 1 << 40]
    dev = torch.device("cuda", 0)
    nt = torch.from_numpy(n).to(dev).contiguous()
    xt = torch.from_numpy(x).to(dev).contiguous()
    saved = _lib.tune_get("demap_hyp")
    try:
        _lib.tune_set("demap_hyp", 1)   # wave-private (default): one wave walks all hypotheses of its tile
        wav = nm.demap_device(nt, xt, B, alpha=0.5).clone()
        _lib.tune_set("demap_hyp", 0)   # one lane per symbol
        per = nm.demap_device(nt, xt, B, alpha=0.5).clone()
    finally:
        _lib.tune_set("demap_hyp", saved)
    torch.cuda.synchronize()
    b = per[:, :B].cpu().numpy()
    a = wav[:, :B].cpu().numpy()
    same = (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), f"{(~same).sum()} LAPPRs differ"
    assert np.isnan(a[bps:2 * bps, :3]).all()
    if bps <= 4:
        onm = O.OracleNoiseMapper(bps, 2.0, nv, cfg)
        for f in (0, 63, 64, B - 1):
            ref = onm.demap_lappr_array(n[2:, f].copy(), x[2:, f].copy()) * 0.5
            assert_bit_exact(a[2 * bps:, f], ref)


# --------------------------------------- F_Y / g / g_inv_search surface (noisemapper.pyx:264-419)
def _case_nm(c):
    import qamr
    import make_golden_cases as MC
    bps, _, probs = MC.NOISE_SEARCH_CASES[c]
    return bps, (None if probs is None else np.array(probs))


@pytest.mark.parametrize("c", range(7))
def test_noise_search_surface_vs_reference(gpu, c):
    """NoiseMapper.F_Y / g / g_inv_search(n_hat, i, y_accuracy) / demap_noise_search through
    libqamr (qr_F_Y_host, qr_g_inv_search_host, qr_map_noise_device) against the reference's
    own outputs: every region, both sign configurations, edge n_hat, y_accuracy 1e-6 / 1e-9 /
    1e-12 (the fast certified search at 1e-9, the verbatim loops otherwise)."""
    import qamr
    import make_golden_cases as MC
    g = golden("noise_search.npz")
    bps, probs = _case_nm(c)
    k = f"c{c}"
    M = 1 << bps
    pa = qamr.PAMAlphabet(bps, 2.0, probs)
    for cfgname in ("base", "alt"):
        cfg = None if cfgname == "base" else MC.alternating(M)
        nm = qamr.NoiseMapper(pa, float(g[f"{k}_noise_var"]), cfg)
        assert_bit_exact(nm.F_Y(g[f"{k}_y"]), g[f"{k}_{cfgname}_F_Y"])
        assert_bit_exact([nm.g(y, i) for y, i in zip(g[f"{k}_y"], g[f"{k}_gi"])], g[f"{k}_{cfgname}_g"])
        nh = g[f"{k}_nhat"]
        for a_i, acc in enumerate(MC.NOISE_SEARCH_ACC):
            ref = g[f"{k}_{cfgname}_ginv_a{a_i}"]
            got = nm.demap_noise_search(np.tile(nh, M), np.repeat(np.arange(M, dtype=np.int64), nh.size), acc)
            assert_bit_exact(got.reshape(M, nh.size), ref)
            # the scalar cpdef on a few points
            for i in (0, M - 1):
                assert_bit_exact([nm.g_inv_search(nh[3], i, acc)], [ref[i, 3]])
        sym = np.full(nh.size, M // 2 - 1 if M > 1 else 0, np.int64)
        assert_bit_exact(nm.demap_noise_search(nh, sym), g[f"{k}_{cfgname}_dns"])


def test_noise_search_random_vs_oracle_and_errors(gpu):
    """Random (n_hat, i) at other accuracies (incl. an exact power of two, where the loop stops
    at width == y_accuracy), fast vs brute search identical, the oracle as checker; out-of-range
    i -> NaN; size / dtype mismatch -> ValueError (noisemapper.pyx:410-411)."""
    import qamr
    from qamr import _lib
    rng = np.random.default_rng(17)
    for bps, nv in ((2, 0.35), (3, 0.8), (4, 0.05)):
        M = 1 << bps
        cfg = rng.integers(0, 2, M).astype(np.uint8)
        nm = _nm(bps, nv, cfg)
        onm = O.OracleNoiseMapper(bps, 2.0, nv, cfg)
        n = rng.uniform(0, 1, 256)
        i = rng.integers(0, M, 256).astype(np.int64)
        for acc in (1e-3, 2.0 ** -20, 1e-9, 3e-11):
            got = nm.demap_noise_search(n, i, acc)
            assert_bit_exact(got, [onm.g_inv_search(a, b, acc) for a, b in zip(n, i)])
        saved = _lib.tune_get("demap_fast")
        try:
            _lib.tune_set("demap_fast", 0)
            brute = nm.demap_noise_search(n, i)
        finally:
            _lib.tune_set("demap_fast", saved)
        assert_bit_exact(nm.demap_noise_search(n, i), brute)
    nm = _nm(2, 1.0)
    assert np.isnan(nm.demap_noise_search(np.array([0.5, 0.5]), np.array([-1, 4], np.int64))).all()
    with pytest.raises(ValueError):
        nm.demap_noise_search(np.zeros(3), np.zeros(2, np.int64))
    with pytest.raises(ValueError):
        nm.demap_noise_search(np.zeros(3, np.float32), np.zeros(3, np.int64))
    with pytest.raises(ValueError):
        nm.F_Y(np.zeros(3, np.int64))
    assert nm.F_Y(np.zeros(0)).size == 0
