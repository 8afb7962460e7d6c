#!/usr/bin/env python3
"""Speed of the CPU restatement (oracle/qamr_oracle.c, the bench's cpu_baseline "port")
relative to the real Cython reference, on 1 core of THIS (build) container and on the same
frames -- BASELINE.md asks for this ratio so that the GPU box's port numbers can be related
to the reference.  Development container only: it imports the reference compiled from its own
sources by `make -C oracle ref` (oracle/_ref, never shipped).

    make -C oracle ref && python3 scripts/cpu_calibrate.py   # -> profiles/cpu_calibration.json

Workloads (bench.py --workload):
  dvbs2_4pam   N=64800 DVB-S2-profile code, 4-PAM 3 dB, decode at 50 iterations
               (Decoder.decode, decoder.pyx:441-455; the construction, decoder.pyx:93-146,
               is one-time and excluded);
  dvbs2_16pam  N=64800, 16-PAM 13 dB: demap (NoiseMapper.demap_lappr_array,
               noisemapper.pyx:544-559) + decode per frame.  The demap is timed on a
               prefix of each frame's symbols and scaled to the frame (its cost is per symbol).
"""
from __future__ import annotations

import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "oracle", "_ref"))

import oracle as O  # noqa: E402  (the C restatement)
from qamr import codes  # noqa: E402
from qamreconciliation.alphabet import PAMAlphabet  # noqa: E402  (the reference build)
from qamreconciliation.decoder import Decoder  # noqa: E402
from qamreconciliation.matrix import Matrix  # noqa: E402
from qamreconciliation.noisemapper import NoiseMapper  # noqa: E402


def cpu_model():
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def frames(bps, snr_db, vid, cid, nfr, seed):
    """Softening inputs (reconciliation.pyx:129-145) from the reference's own classes."""
    M = 1 << bps
    pa = PAMAlphabet(bps, 2.0)
    cfg = np.zeros(M, np.uint8)
    cfg[1::2] = 1
    nv = pa.variance * 10 ** (-snr_db / 10) / 2
    nm = NoiseMapper(pa, nv, cfg)
    mat = Matrix(vid, cid)
    rng = np.random.default_rng(seed)
    S = (int(vid.max()) + 1) // bps
    out = []
    for _ in range(nfr):
        x = rng.choice(M, size=S).astype(np.int64)
        y = np.asarray(pa.index_to_value(x)) + nm.noise_sigma * rng.standard_normal(S)
        xh = np.asarray(nm.hard_decide_index(y), np.int64)
        nh = np.asarray(nm.map_noise(y, xh), np.float64)
        word = np.asarray(pa.demap_symbols_to_bits(xh)).view(np.uint8)
        synd = np.asarray(mat.eval_syndrome(word), np.uint8)
        out.append((x, nh, synd))
    return nm, nv, cfg, out


def timed(fn, *a):
    t0 = time.perf_counter()
    r = fn(*a)
    return r, time.perf_counter() - t0


def main():
    vid, cid = codes.dvbs2_like_half()
    print("building the reference Decoder (O(V E) construction, one-time) ...", flush=True)
    ref_dec, t_build = timed(Decoder, vid, cid)
    port_code = O.OracleCode(vid, cid)
    res = {"cpu": cpu_model(), "cores": 1, "workloads": {},
           "note": "1 thread each; same inputs; the reference is the Cython build of /root/reference "
                   "(oracle/Makefile ref), the port oracle/qamr_oracle.c (gcc -O2 -ffp-contract=off)",
           "reference_decoder_construction_s": t_build}
    for name, bps, snr, nfr, nsym in (("dvbs2_4pam", 2, 3.0, 3, 3000), ("dvbs2_16pam", 4, 13.0, 2, 300)):
        nm, nv, cfg, fr = frames(bps, snr, vid, cid, nfr, seed=7)
        onm = O.OracleNoiseMapper(bps, 2.0, nv, cfg)
        t_ref_dec = t_port_dec = t_ref_dm = t_port_dm = 0.0
        sym_dm = 0
        for x, nh, synd in fr:
            # demap: a prefix of the frame for the reference, the same prefix for the port
            r_dm, t = timed(lambda: np.asarray(nm.demap_lappr_array(nh[:nsym], x[:nsym])))
            t_ref_dm += t
            p_dm, t = timed(onm.demap_lappr_array, nh[:nsym], x[:nsym], 1)
            t_port_dm += t
            sym_dm += nsym
            assert np.array_equal(r_dm.view(np.int64), p_dm.view(np.int64)), "port demap differs from the reference"
            lappr = onm.demap_lappr_array(nh, x, 8)  # the whole frame's LAPPRs (port, 8 threads; not timed)
            (rs, ri, rf), t = timed(ref_dec.decode, lappr, synd, 50)
            t_ref_dec += t
            (ps, pi, pf), t = timed(port_code.decode, lappr, synd, 50)
            t_port_dec += t
            assert (rs, ri) == (ps, pi) and np.array_equal(np.asarray(rf).view(np.int64), pf.view(np.int64)), \
                "port decode differs from the reference"
        S = (int(vid.max()) + 1) // bps
        dec_ref, dec_port = t_ref_dec / nfr, t_port_dec / nfr
        dm_ref, dm_port = t_ref_dm / sym_dm * S, t_port_dm / sym_dm * S
        w = {"frames": nfr, "decode_s_per_frame": {"cython": dec_ref, "port": dec_port},
             "demap_s_per_frame": {"cython": dm_ref, "port": dm_port, "symbols_timed": sym_dm},
             "demap_ratio_port_over_cython": dm_ref / dm_port, "decode_ratio_port_over_cython": dec_ref / dec_port}
        if name == "dvbs2_4pam":  # the bench's 4-PAM step is decode-only (LAPPRs resident)
            w["ratio_port_over_cython"] = dec_ref / dec_port
            w["cython_frames_per_s_per_core"] = 1.0 / dec_ref
        else:  # demap fused into the step
            w["ratio_port_over_cython"] = (dec_ref + dm_ref) / (dec_port + dm_port)
            w["cython_frames_per_s_per_core"] = 1.0 / (dec_ref + dm_ref)
        res["workloads"][name] = w
        print(name, json.dumps(w), flush=True)
    out = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    json.dump(res, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
