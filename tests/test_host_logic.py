"""CPU tests of the host-side logic of the product package (tables, codes,
CSV loader, BER counter, alphabet) against the reference's outputs."""
import os

import numpy as np
import pytest

from conftest import ROOT, assert_bit_exact, golden


def test_alphabet_tables_vs_reference():
    from qamr import PAMAlphabet, generate_table_s_to_b

    g = golden("demap.npz")
    for bps in (1, 2, 3, 4):
        pa = PAMAlphabet(bps, 2.0)
        assert np.array_equal(pa.constellation, g[f"alpha{bps}_constellation"])
        assert np.array_equal(pa.thresholds, g[f"alpha{bps}_thresholds"])
        assert pa.variance == float(g[f"alpha{bps}_variance"])
        assert np.array_equal(pa.s_to_b, g[f"alpha{bps}_s_to_b"])
        assert np.array_equal(generate_table_s_to_b(bps), g[f"alpha{bps}_s_to_b"])
    assert np.array_equal(generate_table_s_to_b(2), [[0, 0], [1, 0], [1, 1], [0, 1]])
    with pytest.raises(ValueError):
        PAMAlphabet(0, 2.0)
    with pytest.raises(ValueError):
        PAMAlphabet(2, 2.0, np.array([0.5, 0.5, 0.5, 0.5]))


@pytest.mark.parametrize("key,bps", [("b1_s20", 1), ("b2_s30", 2), ("b2_s95", 2), ("b4_s130", 4), ("b4_s250", 4)])
def test_noisemapper_host_tables_vs_reference(key, bps):
    from qamr import PAMAlphabet
    from qamr.noisemapper import host_tables

    g = golden("llr_sources.npz")
    pa = PAMAlphabet(bps, 2.0)
    nv = float(g[f"{key}_two_var"]) / 2
    fw, back, bare, ierf = host_tables(pa.constellation, pa.thresholds, pa.probabilities, np.sqrt(nv), bps)
    for cfg in ("base", "alt"):  # the sign configuration does not enter these tables
        # glibc erf/log on both sides, same operation order: bit-exact
        assert np.array_equal(fw, g[f"{key}_{cfg}_fwrd"])
        assert np.array_equal(back, g[f"{key}_{cfg}_back"])
        assert np.array_equal(bare, g[f"{key}_{cfg}_bare"])
        assert np.array_equal(ierf, g[f"{key}_{cfg}_inferf"])
        x = g[f"{key}_x"]
        assert np.array_equal(bare[x].reshape(-1), g[f"{key}_{cfg}_bare_llr_x"])


def test_codes_and_csv(tmp_path):
    from qamr import codes

    vid, cid = codes.dvbs2_like_half()
    assert vid.size == 226799 and codes.code_digest(vid, cid).startswith("22c92f7d6f589b7d")
    deg = np.bincount(cid)
    assert sorted(set(deg.tolist())) == [6, 7] and (deg == 7).sum() == 32399
    v, c = codes.load_edge_csv("/root/reference/test/hamming_7-4.csv") if os.path.exists(
        "/root/reference/test/hamming_7-4.csv") else (golden("hamming.npz")["vid"], golden("hamming.npz")["cid"])
    g = golden("hamming.npz")
    assert np.array_equal(v, g["vid"]) and np.array_equal(c, g["cid"])
    p = tmp_path / "code.csv"
    rv, rc = codes.regular_code(96, seed=1)
    codes.save_edge_csv(str(p), rv, rc)
    v2, c2 = codes.load_edge_csv(str(p))
    assert np.array_equal(v2, rv) and np.array_equal(c2, rc)


def test_count_errors_semantics():
    from qamr.utils import count_errors_from_lappr
    import oracle as O

    rng = np.random.default_rng(0)
    l = rng.standard_normal(1000)
    l[:4] = [0.0, -0.0, np.nan, -1e-300]
    w = rng.integers(0, 2, 1000).astype(np.uint8)
    assert count_errors_from_lappr(l, w) == O.count_errors_from_lappr(l, w)
    with pytest.raises(ValueError):
        count_errors_from_lappr(l, w[:10])


def test_noisemapper_module_functions_vs_reference():
    """The module-level cpdefs F_Z (noisemapper.pyx:66-79) and __view_dist_cut (:82-98) of the
    drop-in equal the reference's outputs bit for bit (tests/golden/module_funcs.npz, from the
    reference built by oracle/Makefile ref)."""
    import qamreconciliation.noisemapper as nmod

    g = golden("module_funcs.npz")
    for c in range(4):
        mu, sigma = g[f"F_Z_{c}_args"]
        assert_bit_exact(nmod.F_Z(g["z"], mu, sigma), g[f"F_Z_{c}"])
    assert_bit_exact(getattr(nmod, "__view_dist_cut")(g["x"]), g["dist_cut"])
    with pytest.raises(ValueError):
        nmod.F_Z(g["z"].astype(np.float32), 0.0, 1.0)
