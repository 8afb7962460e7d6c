"""Generate tests/golden/*.npz from the REFERENCE itself.

Run in the development container only (the reference is not on the GPU box):

    make -C oracle ref                      # builds oracle/_ref from /root/reference sources
    PYTHONPATH=oracle/_ref python3 tests/golden/make_golden.py

Every array stored here is data: inputs and the outputs the reference
(qamreconciliation.decoder / noisemapper / alphabet / matrix, compiled from
/root/reference by oracle/Makefile) returned for them.  No reference source is
stored.  Inputs follow the softening pipeline of sims/reconciliation.pyx:93-147
with seeded numpy RNGs.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle", "_ref"))

import scipy.special  # noqa: E402
from qamreconciliation.alphabet import PAMAlphabet  # noqa: E402  (the reference build)
from qamreconciliation.decoder import Decoder  # noqa: E402
from qamreconciliation.matrix import Matrix  # noqa: E402
from qamreconciliation.noisemapper import NoiseMapper  # noqa: E402

from qamr import codes  # noqa: E402  (synthetic code generators; pure numpy)



def alternating(M):
    cfg = np.zeros(M, np.uint8)
    cfg[1::2] = 1  # sim_reconciliation.py:84-86
    return cfg


def noise_var(pa, snr_db):
    Es = pa.variance
    return Es * (10 ** (-snr_db / 10)) / 2  # reconciliation.pyx:109-110


def softening_inputs(rng, pa, nm, mat, S):
    """reconciliation.pyx:129-145 for one frame (alpha = 1)."""
    x = rng.choice(pa.order, size=S, p=np.asarray(pa.probabilities)).astype(np.int64)
    y = np.asarray(pa.index_to_value(x)) + nm.noise_sigma * rng.standard_normal(S)
    xh = np.asarray(nm.hard_decide_index(y), np.int64)
    nh = np.asarray(nm.map_noise(y, xh), np.float64)
    word = np.asarray(pa.demap_symbols_to_bits(xh)).view(np.uint8)  # cvarray format "c"
    synd = np.asarray(mat.eval_syndrome(word), np.uint8)
    return x, y, xh, nh, word, synd


def gen_hamming():
    import pandas as pd

    df = pd.read_csv("/root/reference/test/hamming_7-4.csv")
    vid = df.vid[1:].to_numpy().astype(np.int64)
    cid = df.cid[1:].to_numpy().astype(np.int64)
    dec = Decoder(vid, cid)
    cases = {
        "correct": (np.array([1.2, -0.8, -1.3, 1.1, -0.4, 0.5, 1.9]), np.array([1, 1, 0], np.uint8)),   # test_decoder.py:238-239
        "one_bit": (np.array([1.05, -1.075, -1.0, 1.1, -0.4, 0.4, -0.2]), np.array([1, 1, 0], np.uint8)),  # :251-252
    }
    out = {"vid": vid, "cid": cid}
    rng = np.random.default_rng(7)
    extra_l = rng.standard_normal((32, 7)) * 1.5
    extra_s = rng.integers(0, 2, (32, 3)).astype(np.uint8)
    for name, (l, s) in cases.items():
        ok, it, r = dec.decode(l, s, 20)
        out[f"{name}_lappr"], out[f"{name}_synd"] = l, s
        out[f"{name}_success"], out[f"{name}_iters"], out[f"{name}_final"] = ok, it, np.asarray(r)
    fin = np.empty_like(extra_l)
    succ = np.empty(32, np.uint8)
    its = np.empty(32, np.int32)
    for f in range(32):
        ok, it, r = dec.decode(extra_l[f], extra_s[f], 20)
        fin[f], succ[f], its[f] = np.asarray(r), ok, it
    out.update(rand_lappr=extra_l, rand_synd=extra_s, rand_final=fin, rand_success=succ, rand_iters=its)
    # max_iterations edge cases on the one-bit-error word
    for mi in (0, 1, 2):
        ok, it, r = dec.decode(cases["one_bit"][0], cases["one_bit"][1], mi)
        out[f"maxit{mi}_success"], out[f"maxit{mi}_iters"], out[f"maxit{mi}_final"] = ok, it, np.asarray(r)
    np.savez_compressed(os.path.join(HERE, "hamming.npz"), **out)


def gen_node_rules():
    """test_decoder.py:132-220 graph; process_* outputs on seeded messages."""
    vid = np.array([0, 1, 3, 1, 2, 1, 3, 4], np.int64)
    cid = np.array([0, 0, 0, 1, 1, 2, 2, 2], np.int64)
    dec = Decoder(vid, cid)
    rng = np.random.default_rng(11)
    out = {"vid": vid, "cid": cid}
    for t in range(4):
        c2v = rng.standard_normal(8) * 2
        v2c = rng.standard_normal(8) * 2
        l = rng.standard_normal(5)
        synd = rng.integers(0, 2, 3).astype(np.uint8)
        out[f"t{t}_c2v_in"], out[f"t{t}_v2c_in"], out[f"t{t}_lappr"], out[f"t{t}_synd"] = c2v, v2c, l, synd
        for v in range(5):
            a, b, u = c2v.copy(), v2c.copy(), np.zeros(5)
            dec.process_var_node(v, l, a, b, u)
            out[f"t{t}_var{v}_v2c"], out[f"t{t}_var{v}_upd"] = b, u
        for c in range(3):
            a, b = c2v.copy(), v2c.copy()
            dec.process_check_node(c, synd, a, b)
            out[f"t{t}_chk{c}_c2v"] = a
    np.savez_compressed(os.path.join(HERE, "node_rules.npz"), **out)


def gen_reg1008():
    vid, cid = codes.regular_code(1008)
    dec, mat = Decoder(vid, cid), Matrix(vid, cid)
    pa = PAMAlphabet(2, 2.0)
    out = {"vid": vid, "cid": cid}
    for snr in (2.0, 4.0, 6.0):
        nv = noise_var(pa, snr)
        nm = NoiseMapper(pa, nv, alternating(pa.order))
        rng = np.random.default_rng(int(10 * snr) + 2)
        F = 16
        L = np.empty((F, 1008)); Sy = np.empty((F, 504), np.uint8); W = np.empty((F, 1008), np.uint8)
        Fin = np.empty((F, 1008)); Su = np.empty(F, np.uint8); It = np.empty(F, np.int32)
        for f in range(F):
            x, y, xh, nh, word, synd = softening_inputs(rng, pa, nm, mat, 504)
            lappr = np.asarray(nm.demap_lappr_array(nh, x))
            ok, it, r = dec.decode(lappr, synd, 50)
            L[f], Sy[f], W[f], Fin[f], Su[f], It[f] = lappr, synd, word, np.asarray(r), ok, it
        k = f"snr{int(snr)}"
        out.update({f"{k}_lappr": L, f"{k}_synd": Sy, f"{k}_word": W, f"{k}_final": Fin,
                    f"{k}_success": Su, f"{k}_iters": It, f"{k}_noise_var": nv})
    np.savez_compressed(os.path.join(HERE, "reg1008.npz"), **out)


def gen_demap():
    out = {}
    for bps, snrs, S in ((2, (3.0, 4.0, 9.5), 400), (4, (13.0, 14.5, 25.0), 60)):
        pa = PAMAlphabet(bps, 2.0)
        for snr in snrs:
            nv = noise_var(pa, snr)
            cfg = alternating(pa.order)
            nm = NoiseMapper(pa, nv, cfg)
            rng = np.random.default_rng(1000 * bps + int(10 * snr))
            x = rng.choice(pa.order, size=S).astype(np.int64)
            y = np.asarray(pa.index_to_value(x)) + nm.noise_sigma * rng.standard_normal(S)
            xh = np.asarray(nm.hard_decide_index(y), np.int64)
            nh = np.asarray(nm.map_noise(y, xh), np.float64)
            la = np.asarray(nm.demap_lappr_array(nh, x))
            k = f"b{bps}_s{int(10 * snr)}"
            out.update({f"{k}_noise_var": nv, f"{k}_cfg": cfg, f"{k}_x": x, f"{k}_y": y, f"{k}_xhat": xh,
                        f"{k}_nhat": nh, f"{k}_lappr": la,
                        f"{k}_Fthr": np.asarray(nm.F_Y_thresholds), f"{k}_dF": np.asarray(nm.delta_F_Y),
                        f"{k}_word": np.asarray(pa.demap_symbols_to_bits(xh)).view(np.uint8).copy()})
            # base (all-zero) sign configuration on a few symbols too
            nm0 = NoiseMapper(pa, nv)
            out[f"{k}_lappr_base"] = np.asarray(nm0.demap_lappr_array(nh[:20], x[:20]))
            out[f"{k}_nhat_base"] = np.asarray(nm0.map_noise(y[:20], xh[:20]), np.float64)
    # alphabet tables
    for bps in (1, 2, 3, 4):
        pa = PAMAlphabet(bps, 2.0)
        out[f"alpha{bps}_constellation"] = np.asarray(pa.constellation)
        out[f"alpha{bps}_thresholds"] = np.asarray(pa.thresholds)
        out[f"alpha{bps}_variance"] = pa.variance
        out[f"alpha{bps}_s_to_b"] = np.asarray(pa.s_to_b)
    # scipy.special.erf points (the reference's erf, noisemapper.pyx:67)
    rng = np.random.default_rng(99)
    ex = np.concatenate([rng.normal(0, 3, 4000), rng.uniform(-30, 30, 2000), rng.uniform(-1.05, 1.05, 2000),
                         np.array([0.0, -0.0, 1.0, -1.0, 8.0, -8.0, 26.6, 27.0, np.inf, -np.inf])])
    out["erf_x"], out["erf_y"] = ex, scipy.special.erf(ex)
    np.savez_compressed(os.path.join(HERE, "demap.npz"), **out)


def gen_dvbs2():
    """Two N=64800 frames through the reference (demap + decode), stored compactly."""
    vid, cid = codes.dvbs2_like_half()
    t = time.time()
    dec, mat = Decoder(vid, cid), Matrix(vid, cid)
    print(f"  reference Decoder.__cinit__ N=64800: {time.time() - t:.1f} s", flush=True)
    out = {"digest": codes.code_digest(vid, cid)}
    pa = PAMAlphabet(2, 2.0)
    for snr in (3.0, 4.0):
        nv = noise_var(pa, snr)
        nm = NoiseMapper(pa, nv, alternating(4))
        rng = np.random.default_rng(int(10 * snr) + 2)
        x, y, xh, nh, word, synd = softening_inputs(rng, pa, nm, mat, 32400)
        t = time.time()
        lappr = np.asarray(nm.demap_lappr_array(nh, x))
        td = time.time() - t
        t = time.time()
        ok, it, r = dec.decode(lappr, synd, 50)
        tc = time.time() - t
        r = np.asarray(r)
        print(f"  snr {snr}: demap {td:.1f} s, decode {tc:.2f} s, success={ok} iters={it}", flush=True)
        k = f"snr{int(10 * snr)}"
        idx = np.random.default_rng(5).choice(64800, 4096, replace=False)
        out.update({f"{k}_x": x.astype(np.int8), f"{k}_nhat": nh, f"{k}_lappr": lappr,
                    f"{k}_synd_packed": np.packbits(synd), f"{k}_word_packed": np.packbits(word),
                    f"{k}_success": ok, f"{k}_iters": it, f"{k}_hard_packed": np.packbits(r < 0),
                    f"{k}_sample_idx": idx, f"{k}_sample_final": r[idx],
                    f"{k}_noise_var": nv, f"{k}_ref_decode_s": tc, f"{k}_ref_demap_s": td})
    np.savez_compressed(os.path.join(HERE, "dvbs2.npz"), **out)


def _demap_chunk(args):
    """One worker's share of a reference demap (symbols are independent:
    noisemapper.pyx:544-559 loops demap_lappr over them)."""
    bps, nv, nh, x = args
    pa = PAMAlphabet(bps, 2.0)
    nm = NoiseMapper(pa, nv, alternating(pa.order))
    return np.asarray(nm.demap_lappr_array(nh, x)).copy()


def gen_dvbs2_16pam():
    """configs[3] pinned to the reference itself: two N=64800 16-PAM frames (13.0 dB, all
    50 iterations; 14.5 dB, converging) through the reference's demap_lappr_array and
    Decoder.decode (the path of sims/reconciliation.pyx:129-147).  The reference demap
    (~95 s per frame on one core) runs on symbol chunks in a process pool: every symbol's
    LAPPRs come from the same demap_lappr call as in the sequential loop."""
    import multiprocessing as mp

    vid, cid = codes.dvbs2_like_half()
    t = time.time()
    dec, mat = Decoder(vid, cid), Matrix(vid, cid)
    print(f"  reference Decoder.__cinit__ N=64800: {time.time() - t:.1f} s", flush=True)
    out = {"digest": codes.code_digest(vid, cid)}
    pa = PAMAlphabet(4, 2.0)
    nproc = min(8, os.cpu_count() or 1)
    for snr in (13.0, 14.5):
        nv = noise_var(pa, snr)
        nm = NoiseMapper(pa, nv, alternating(16))
        rng = np.random.default_rng(int(10 * snr) + 4)
        x, y, xh, nh, word, synd = softening_inputs(rng, pa, nm, mat, 16200)
        t = time.time()
        parts = np.array_split(np.arange(16200), 4 * nproc)
        with mp.get_context("fork").Pool(nproc) as pool:
            chunks = pool.map(_demap_chunk, [(4, nv, nh[p].copy(), x[p].copy()) for p in parts])
        lappr = np.concatenate(chunks)
        td = time.time() - t
        # a sequential spot check: the pool returned the reference's own values
        assert np.array_equal(np.asarray(nm.demap_lappr_array(nh[:40], x[:40])).view(np.int64),
                              lappr[:160].view(np.int64))
        t = time.time()
        ok, it, r = dec.decode(lappr, synd, 50)
        tc = time.time() - t
        r = np.asarray(r)
        print(f"  16-PAM snr {snr}: demap {td:.1f} s ({nproc} procs), decode {tc:.2f} s, success={ok} "
              f"iters={it}", flush=True)
        k = f"snr{int(10 * snr)}"
        out.update({f"{k}_x": x.astype(np.int8), f"{k}_nhat": nh, f"{k}_lappr": lappr,
                    f"{k}_synd_packed": np.packbits(synd), f"{k}_word_packed": np.packbits(word),
                    f"{k}_success": ok, f"{k}_iters": it, f"{k}_hard_packed": np.packbits(r < 0),
                    f"{k}_final": r, f"{k}_noise_var": nv, f"{k}_ref_decode_s": tc,
                    f"{k}_ref_demap_s": td, f"{k}_ref_demap_procs": nproc})
    np.savez_compressed(os.path.join(HERE, "dvbs2_16pam.npz"), **out)


def gen_pam16_nan():
    """16-PAM at 25 dB on reg-(3,6) N=1008: +-inf LAPPRs from the demap, then the
    reference's decode behaviour on them (inf -> NaN)."""
    vid, cid = codes.regular_code(1008)
    dec, mat = Decoder(vid, cid), Matrix(vid, cid)
    pa = PAMAlphabet(4, 2.0)
    nv = noise_var(pa, 25.0)
    nm = NoiseMapper(pa, nv, alternating(16))
    rng = np.random.default_rng(250)
    out = {"noise_var": nv}
    for f in range(3):
        x, y, xh, nh, word, synd = softening_inputs(rng, pa, nm, mat, 252)
        lappr = np.asarray(nm.demap_lappr_array(nh, x))
        ok, it, r = dec.decode(lappr, synd, 50)
        out.update({f"f{f}_x": x, f"f{f}_nhat": nh, f"f{f}_lappr": lappr, f"f{f}_synd": synd,
                    f"f{f}_success": ok, f"f{f}_iters": it, f"f{f}_final": np.asarray(r)})
        print(f"  pam16 25dB frame {f}: inf={np.isinf(lappr).sum()} success={ok} iters={it} "
              f"nan_out={np.isnan(np.asarray(r)).sum()}", flush=True)
    np.savez_compressed(os.path.join(HERE, "pam16_25db.npz"), **out)


def gen_llr_sources():
    """Direct-reconciliation LAPPRs (sims/reconciliation.pyx:25-65 via the cpdef
    y_to_lappr_grey_array) and the NoiseMapper host tables (noisemapper.pyx:166-235)."""
    from sims.reconciliation import y_to_lappr_grey_array

    out = {}
    for bps, snrs in ((1, (2.0,)), (2, (3.0, 9.5)), (4, (13.0, 25.0))):
        pa = PAMAlphabet(bps, 2.0)
        for snr in snrs:
            k = f"b{bps}_s{int(10 * snr)}"
            Es = pa.variance
            two_var = Es * (10 ** (-snr / 10))
            nv = two_var / 2
            rng = np.random.default_rng(77 + bps)
            x = rng.choice(pa.order, size=200).astype(np.int64)
            y = np.asarray(pa.index_to_value(x)) + np.sqrt(nv) * rng.standard_normal(200)
            out[f"{k}_two_var"], out[f"{k}_y"] = two_var, y
            out[f"{k}_direct"] = np.asarray(y_to_lappr_grey_array(y, pa, two_var))
            for cfgname, cfg in (("base", None), ("alt", alternating(pa.order))):
                nm = NoiseMapper(pa, nv, cfg) if cfg is not None else NoiseMapper(pa, nv)
                out[f"{k}_{cfgname}_fwrd"] = np.asarray(nm.fwrd_transition_probability)
                out[f"{k}_{cfgname}_back"] = np.asarray(nm.back_transition_probability)
                out[f"{k}_{cfgname}_bare"] = np.asarray(nm.bare_llr_table)
                out[f"{k}_{cfgname}_inferf"] = np.asarray(nm.inf_erf_table)
                out[f"{k}_{cfgname}_bare_llr_x"] = np.asarray(nm.bare_llr(x))
            out[f"{k}_x"] = x
    np.savez_compressed(os.path.join(HERE, "llr_sources.npz"), **out)


from make_golden_cases import NOISE_SEARCH_ACC, NOISE_SEARCH_CASES  # noqa: E402


def gen_noise_search():
    """The cpdef surface of NoiseMapper around the search (noisemapper.pyx:264-345, 407-419):
    F_Y on a y grid, g(y, i), and g_inv_search(n_hat, i, y_accuracy) for every decision
    region, both sign configurations, edge n_hat (0, 1, 1/2, subnormal, 1 - 2^-53 ...) and
    y_accuracy in {1e-6, 1e-9, 1e-12}."""
    out = {}
    for c, (bps, snr, probs) in enumerate(NOISE_SEARCH_CASES):
        pa = PAMAlphabet(bps, 2.0, None if probs is None else np.array(probs))
        nv = noise_var(pa, snr)
        rng = np.random.default_rng(500 + c)
        k = f"c{c}"
        out[f"{k}_noise_var"] = nv
        M = pa.order
        edge = np.array([0.0, 1.0, 0.5, 5e-324, 1e-300, 1e-17, 1e-9, 1 - 2 ** -53, 0.25, 0.999999])
        nh = np.concatenate([edge, rng.uniform(0, 1, 14)])
        ii = np.arange(M, dtype=np.int64)
        # y grid through every region and far into both tails
        y = np.concatenate([np.linspace(pa.constellation[0] * 1.6, pa.constellation[-1] * 1.6, 41),
                            rng.normal(0, 2 * M, 24), np.array([0.0, -0.0, 1e3, -1e3, 40.0, -40.0])])
        out[f"{k}_y"] = y
        gi = rng.integers(0, M, y.size).astype(np.int64)
        out[f"{k}_gi"] = gi
        for cfgname, cfg in (("base", None), ("alt", alternating(M))):
            nm = NoiseMapper(pa, nv, cfg) if cfg is not None else NoiseMapper(pa, nv)
            out[f"{k}_{cfgname}_F_Y"] = np.asarray(nm.F_Y(y.copy()))
            out[f"{k}_{cfgname}_g"] = np.array([nm.g(float(yy), int(i)) for yy, i in zip(y, gi)])
            for a_i, acc in enumerate(NOISE_SEARCH_ACC):
                res = np.array([[nm.g_inv_search(float(n), int(i), acc) for n in nh] for i in ii])
                out[f"{k}_{cfgname}_ginv_a{a_i}"] = res
            out[f"{k}_{cfgname}_dns"] = np.asarray(nm.demap_noise_search(nh.copy(), np.full(nh.size, M // 2 - 1 if M > 1 else 0, np.int64)))
        out[f"{k}_nhat"] = nh
    np.savez_compressed(os.path.join(HERE, "noise_search.npz"), **out)


def gen_module_funcs():
    """The module-level cpdefs of noisemapper.pyx: F_Z(z, mu, sigma) (:66-79) and
    __view_dist_cut(x) (:82-98) on edge and random points."""
    import qamreconciliation.noisemapper as nmod

    rng = np.random.default_rng(77)
    z = np.concatenate([np.array([0.0, -0.0, 1.0, -1.0, 1e-300, -1e300, 1e300, 40.0, -40.0, np.inf, -np.inf, np.nan]),
                        rng.normal(0, 3, 40)])
    out = {"z": z}
    for c, (mu, sigma) in enumerate([(0.0, 1.0), (1.5, 0.3), (-2.0, 4.0), (0.0, 1e-3)]):
        out[f"F_Z_{c}"] = np.asarray(nmod.F_Z(z.copy(), mu, sigma))
        out[f"F_Z_{c}_args"] = np.array([mu, sigma])
    x = np.concatenate([np.array([-1.0, -0.0, 0.0, 1e-300, 0.5, 1 - 2 ** -53, 1.0, 1.5, np.inf, -np.inf, np.nan]),
                        rng.uniform(-0.5, 1.5, 30)])
    out["x"] = x
    out["dist_cut"] = np.asarray(getattr(nmod, "__view_dist_cut")(x.copy()))
    np.savez_compressed(os.path.join(HERE, "module_funcs.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["hamming", "node_rules", "reg1008", "demap", "pam16_nan", "llr_sources", "dvbs2",
                             "dvbs2_16pam", "noise_search", "module_funcs"]
    for w in which:
        t = time.time()
        print(f"[golden] {w}", flush=True)
        globals()[f"gen_{w}"]()
        print(f"[golden] {w} done in {time.time() - t:.1f} s", flush=True)
