"""GPU parity tests of the decoder: libqamr (HIP, gfx950) against the reference's
golden outputs and the oracle.  With the default (strict) arithmetic every output
-- success flags, iteration counts, hard decisions and the final LAPPRs -- must be
bit-exact (conftest.assert_bit_exact)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_bit_exact, golden

import oracle as O

pytestmark = pytest.mark.gpu


def _decoder(vid, cid):
    import qamr
    return qamr.Decoder(np.asarray(vid, np.int64), np.asarray(cid, np.int64))


def test_hamming_reference_unit_tests(gpu):
    g = golden("hamming.npz")
    dec = _decoder(g["vid"], g["cid"])
    assert (dec.vnum, dec.cnum, dec.ednum) == (7, 3, 12)
    # test_decoder.py:237-248
    ok, it, r = dec.decode(g["correct_lappr"], g["correct_synd"], 20)
    assert ok and it == 0 and (r != g["correct_lappr"]).sum() == 0
    # test_decoder.py:250-266
    ok, it, r = dec.decode(g["one_bit_lappr"], g["one_bit_synd"], 20)
    assert ok and it <= 20
    assert np.array_equal((np.asarray(r) < 0).astype(int), [0, 1, 1, 0, 1, 0, 0])
    assert it == int(g["one_bit_iters"])
    assert_bit_exact(r, g["one_bit_final"])
    for mi in (0, 1, 2):
        ok, it, r = dec.decode(g["one_bit_lappr"], g["one_bit_synd"], mi)
        assert (ok, it) == (int(g[f"maxit{mi}_success"]), int(g[f"maxit{mi}_iters"]))
        assert_bit_exact(r, g[f"maxit{mi}_final"])
    s, i, f = dec.decode_batch(g["rand_lappr"], g["rand_synd"], 20)
    assert np.array_equal(s, g["rand_success"]) and np.array_equal(i, g["rand_iters"])
    assert_bit_exact(f, g["rand_final"])


def test_construction_surface(gpu):
    # test_decoder.py:8-128
    dec = _decoder([0, 1, 1, 2], [0, 0, 1, 1])
    assert (dec.cnum, dec.vnum, dec.ednum) == (2, 3, 4)
    synd0, synd1 = np.array([1, 1], np.uint8), np.array([0, 1], np.uint8)
    for w in np.array([[1, 0, 1], [0, 1, 0]], np.uint8):
        assert dec.check_word(w, synd0) and not dec.check_word(w, synd1)
        for c in (0, 1):
            assert dec.check_synd_node(c, w, synd0)
            assert not dec.check_synd_node(0, w, synd1) if c == 0 else dec.check_synd_node(1, w, synd1)
    for w in np.array([[0, 0, 1], [1, 1, 0]], np.uint8):
        assert dec.check_word(w, synd1) and not dec.check_word(w, synd0)
    assert dec.check_lappr(np.array([-3.4, 0.8, -0.1]), synd0)
    assert not dec.check_lappr(np.array([-3.4, 0.8, -0.1]), synd1)
    assert dec.check_lappr(np.array([-0.77, -0.8, 0.98]), synd1)
    assert not dec.check_lappr(np.array([-0.77, -0.8, 0.98]), synd0)
    with pytest.raises(ValueError):
        dec.check_lappr(np.zeros(4), synd0)
    with pytest.raises(ValueError):
        _decoder([0, 1, 2], [0, 0])


def test_node_rules(gpu):
    g = golden("node_rules.npz")
    dec = _decoder(g["vid"], g["cid"])
    for t in range(4):
        for v in range(5):
            c2v, v2c, u = g[f"t{t}_c2v_in"].copy(), g[f"t{t}_v2c_in"].copy(), np.zeros(5)
            dec.process_var_node(v, g[f"t{t}_lappr"], c2v, v2c, u)
            # additions/subtractions only: bit-exact
            assert np.array_equal(v2c, g[f"t{t}_var{v}_v2c"]) and np.array_equal(u, g[f"t{t}_var{v}_upd"])
        for c in range(3):
            c2v, v2c = g[f"t{t}_c2v_in"].copy(), g[f"t{t}_v2c_in"].copy()
            assert dec.process_check_node(c, g[f"t{t}_synd"], c2v, v2c) == 0
            assert_bit_exact(c2v, g[f"t{t}_chk{c}_c2v"])
    # test_decoder.py:189-220 analytic form
    rng = np.random.default_rng(3)
    c2v, v2c = rng.standard_normal(8), rng.standard_normal(8)
    s = np.array([0, 1, 0], np.uint8)
    dec.process_check_node(1, s, c2v, v2c)
    assert abs(c2v[3] - (-2 * v2c[4] / 2)) <= abs(c2v[3]) * 1e-6
    dec.process_check_node(2, s, c2v, v2c)
    ref = 2 * np.arctanh(np.tanh(v2c[6] / 2) * np.tanh(v2c[7] / 2))
    assert abs(c2v[5] - ref) <= abs(c2v[5]) * 1e-6


def test_reg1008_golden_frames(gpu):
    g = golden("reg1008.npz")
    dec = _decoder(g["vid"], g["cid"])
    for k in ("snr2", "snr4", "snr6"):
        s, i, f = dec.decode_batch(g[f"{k}_lappr"], g[f"{k}_synd"], 50)
        assert np.array_equal(s, g[f"{k}_success"]), k
        assert np.array_equal(i, g[f"{k}_iters"]), k
        assert np.array_equal(f < 0, g[f"{k}_final"] < 0), k
        assert_bit_exact(f, g[f"{k}_final"])


def test_reg1008_batch_vs_oracle_random(gpu):
    """Fresh seeded inputs (B = 200: not a multiple of 64) through both paths."""
    from qamr import codes

    vid, cid = codes.regular_code(1008)
    dec = _decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    rng = np.random.default_rng(42)
    B = 200
    sig = rng.uniform(0.55, 1.0, B)[:, None]
    word = rng.integers(0, 2, (B, 1008)).astype(np.uint8)
    synd = np.stack([orc.eval_syndrome(w) for w in word])
    llr = 2 / sig ** 2 * ((1 - 2.0 * word) + sig * rng.standard_normal((B, 1008)))
    s1, i1, f1 = dec.decode_batch(llr, synd, 50)
    s2, i2, f2 = orc.decode_batch(llr, synd, 50)
    assert np.array_equal(s1, s2) and np.array_equal(i1, i2)
    assert_bit_exact(f1, f2)
    assert 0 < s1.sum() < B  # both converging and failing frames exercised


def test_edge_cases(gpu):
    from qamr import codes

    vid, cid = codes.regular_code(96, seed=3)
    dec = _decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    rng = np.random.default_rng(9)
    l = rng.standard_normal((5, 96)) * 2
    l[0, :5] = [-0.0, 0.0, np.inf, -np.inf, 1e-310]   # signed zeros, infinities, subnormal
    l[1, 3] = np.nan
    synd = rng.integers(0, 2, (5, 48)).astype(np.uint8)
    for mi in (-3, 0, 1, 7, 50):
        s1, i1, f1 = dec.decode_batch(l, synd, mi)
        for f in range(5):
            ok, it, r = orc.decode(l[f], synd[f], mi)
            assert (s1[f], i1[f]) == (ok, it), (mi, f)
            assert_bit_exact(f1[f], r)
    # degree-1 check rejected (UB in the reference)
    with pytest.raises(ValueError):
        _decoder([0, 1, 2], [0, 0, 1])
    # parallel edges are processed like the reference does
    vid2 = np.array([0, 0, 1, 2, 1, 2, 3, 3], np.int64)
    cid2 = np.array([0, 0, 0, 1, 1, 1, 2, 2], np.int64)
    d2, o2 = _decoder(vid2, cid2), O.OracleCode(vid2, cid2)
    ll = np.array([0.3, -1.2, 0.4, 0.9])
    for sy in ([0, 1, 0], [1, 1, 1], [0, 0, 1]):
        sy = np.array(sy, np.uint8)
        a, b = dec_one(d2, ll, sy), o2.decode(ll, sy, 30)
        assert a[:2] == b[:2]
        assert_bit_exact(a[2], b[2])


def dec_one(d, l, s):
    ok, it, r = d.decode(l, s, 30)
    return ok, it, r


def test_dvbs2_golden_frames(gpu):
    if not os.path.exists(os.path.join(GOLDEN, "dvbs2.npz")):
        pytest.skip("dvbs2.npz not generated")
    from qamr import codes

    g = golden("dvbs2.npz")
    vid, cid = codes.dvbs2_like_half()
    dec = _decoder(vid, cid)
    L = np.stack([g["snr30_lappr"], g["snr40_lappr"]])
    S = np.stack([np.unpackbits(g[f"{k}_synd_packed"])[:32400] for k in ("snr30", "snr40")])
    s, i, f = dec.decode_batch(L, S, 50)
    for b, k in enumerate(("snr30", "snr40")):
        assert s[b] == int(g[f"{k}_success"]) and i[b] == int(g[f"{k}_iters"])
        assert np.array_equal(np.packbits(f[b] < 0), g[f"{k}_hard_packed"])
        assert_bit_exact(f[b][g[f"{k}_sample_idx"]], g[f"{k}_sample_final"])


def test_device_api_layout_and_properties(gpu):
    """decode_device on HBM tensors: frames are independent (permuting frames
    permutes results) and the result equals the host path."""
    import torch
    from qamr import codes
    from qamr.pipeline import leading_dim

    vid, cid = codes.regular_code(1008)
    dec = _decoder(vid, cid)
    g = golden("reg1008.npz")
    L = np.concatenate([g[f"{k}_lappr"] for k in ("snr2", "snr4", "snr6")])
    S = np.concatenate([g[f"{k}_synd"] for k in ("snr2", "snr4", "snr6")])
    B = L.shape[0]
    ld = leading_dim(B)
    dev = torch.device("cuda", 0)
    lt = torch.zeros((1008, ld), dtype=torch.float64, device=dev)
    st = torch.zeros((504, ld), dtype=torch.uint8, device=dev)
    lt[:, :B] = torch.from_numpy(L.T.copy()).to(dev)
    st[:, :B] = torch.from_numpy(S.T.copy()).to(dev)
    fin, succ, its = dec.decode_device(lt, st, B, 50)
    torch.cuda.synchronize()
    s_h, i_h, f_h = dec.decode_batch(L, S, 50)
    assert np.array_equal(succ.cpu().numpy(), s_h) and np.array_equal(its.cpu().numpy(), i_h)
    assert np.array_equal(fin[:, :B].cpu().numpy().T, f_h)
    perm = np.random.default_rng(0).permutation(B)
    s_p, i_p, f_p = dec.decode_batch(L[perm], S[perm], 50)
    assert np.array_equal(s_p, s_h[perm]) and np.array_equal(i_p, i_h[perm]) and np.array_equal(f_p, f_h[perm])


def test_large_magnitude_inputs_bit_exact(gpu):
    """The strict arithmetic (the only one) is bit-identical to the oracle also on frames
    whose check inputs are large (|LLR| in the hundreds and thousands, inf).  Results never
    depend on which frames share a wavefront (permuting frames permutes results bit for bit)."""
    from qamr import _lib, codes

    vid, cid = codes.regular_code(1008)
    dec = _decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    rng = np.random.default_rng(7)
    B = 192
    sig = rng.uniform(0.55, 1.0, B)[:, None]
    word = rng.integers(0, 2, (B, 1008)).astype(np.uint8)
    synd = np.stack([orc.eval_syndrome(w) for w in word])
    llr = 2 / sig ** 2 * ((1 - 2.0 * word) + sig * rng.standard_normal((B, 1008)))
    big = rng.choice(B, 40, replace=False)
    llr[big[:20]] *= 150.0                                   # |LLR| in the hundreds..thousands
    llr[big[20:], :30] *= 1e4                                 # a few huge inputs per frame
    llr[big[0], 5] = np.inf
    s2, i2, f2 = orc.decode_batch(llr, synd, 50)
    with pytest.raises(ValueError):  # the approximate arithmetics are gone (unknown knob)
        _lib.tune_set("math", 1)
    s1, i1, f1 = dec.decode_batch(llr, synd, 50)
    assert np.array_equal(s1, s2) and np.array_equal(i1, i2)
    assert_bit_exact(f1, f2)
    perm = rng.permutation(B)
    s_p, i_p, f_p = dec.decode_batch(llr[perm], synd[perm], 50)
    assert np.array_equal(s_p, s2[perm]) and np.array_equal(i_p, i2[perm])
    assert_bit_exact(f_p, f1[perm])


def test_decode_device_graph_capture(gpu):
    """The batched decode (every schedule, incl. the default two-stream one whose second
    stream forks from and joins the caller's stream through events) is capturable in a
    HIP graph: the replay reproduces the eager decode bit for bit."""
    import torch
    from qamr import _lib, codes

    vid, cid = codes.regular_code(1008)
    dec = _decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    rng = np.random.default_rng(21)
    B = 512
    sig = rng.uniform(0.55, 0.9, B)[:, None]
    word = rng.integers(0, 2, (B, 1008)).astype(np.uint8)
    synd = np.stack([orc.eval_syndrome(w) for w in word])
    llr = 2 / sig ** 2 * ((1 - 2.0 * word) + sig * rng.standard_normal((B, 1008)))
    L = torch.from_numpy(llr.T.copy()).cuda()
    S = torch.from_numpy(synd.T.copy()).cuda()
    saved = _lib.tune_get("split")
    try:
        for split in (3, 2, 1):
            _lib.tune_set("split", split)
            ref = [x.clone() for x in dec.decode_device(L, S, B, 30)]  # eager (also allocates)
            fin = torch.full_like(L, np.nan)
            succ = torch.zeros(B, dtype=torch.uint8, device="cuda")
            its = torch.zeros(B, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                dec.decode_device(L, S, B, 30, fin, succ, its)
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(succ, ref[1]) and torch.equal(its, ref[2]), split
            assert torch.equal(fin.view(torch.int64), ref[0].view(torch.int64)), split
    finally:
        _lib.tune_set("split", saved)


def test_strict_clamp_paths(gpu):
    """The strict check sweep picks its clamp of the h arguments per batch (decoder.hip
    QR_STRICT_FINITE): every LAPPR below 2^e (e = 1000 - (max_it + 2) log2(dv_max + 1)) ->
    max(-|t|, -700); otherwise (inf, NaN, or finite but huge) the NaN-preserving clamp.
    Both are bit-identical to the reference's h (decoder.pyx:41-45) on arguments far beyond
    the 37.5 where h becomes 0, in batches that differ only in one frame."""
    from qamr import codes

    vid, cid = codes.regular_code(1008)
    dec = _decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    rng = np.random.default_rng(11)
    B = 128
    sig = rng.uniform(0.55, 1.0, B)[:, None]
    word = rng.integers(0, 2, (B, 1008)).astype(np.uint8)
    synd = np.stack([orc.eval_syndrome(w) for w in word])
    llr = 2 / sig ** 2 * ((1 - 2.0 * word) + sig * rng.standard_normal((B, 1008)))
    llr[:40] *= rng.choice([300.0, 1e3, 1e6], (40, 1))          # box-plus arguments >> 700
    llr[40:50, :60] *= 1e12
    cases = {"bounded": llr.copy()}
    x = llr.copy(); x[3, 7] = np.inf; cases["inf"] = x
    x = llr.copy(); x[5, 9] = np.nan; cases["nan"] = x
    x = llr.copy(); x[60, 11] = 1e300; cases["huge"] = x           # finite, above the bound
    for name, l in cases.items():
        s1, i1, f1 = dec.decode_batch(l, synd, 50)
        s2, i2, f2 = orc.decode_batch(l, synd, 50)
        assert np.array_equal(s1, s2) and np.array_equal(i1, i2), name
        assert_bit_exact(f1, f2)
    # max_it = 600: (600 + 2) log2(dv_max + 1) > 1000, the flag is cleared without a test
    # (the decode keeps the NaN-preserving clamp whatever the inputs)
    l = llr[:64].copy()
    s1, i1, f1 = dec.decode_batch(l, synd[:64], 600)
    s2, i2, f2 = orc.decode_batch(l, synd[:64], 600)
    assert np.array_equal(s1, s2) and np.array_equal(i1, i2)
    assert_bit_exact(f1, f2)
