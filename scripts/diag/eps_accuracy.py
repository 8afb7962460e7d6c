"""Accuracy of the exp-domain check update vs the oracle on the bench workloads.

    python scripts/diag/eps_accuracy.py [--frames 96]

For each (PAM order, SNR) operating point: B frames generated on the GPU by the
softening pipeline, decoded by the oracle (reference arithmetic, CPU) and by
libqamr with math=0 (strict, glibc-exact), 1 (table h) and 2 (exp domain) at several eps_max.  Prints
success/iteration/hard-decision agreement, the worst LAPPR error in units of the
north-star tolerance (1e-6 |ref| + 1e-9), and the share of lanes of the
checks' input magnitudes above each eps_max (from the oracle's final LAPPRs).
Diagnostic only (oracle = checker)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "qam-reconciliation_amd"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
import qamr  # noqa: E402
from qamr import _lib, codes  # noqa: E402
from qamr.pipeline import SofteningPipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=96)
    ap.add_argument("--points", default="2:3.0,2:4.0,4:13.0,4:14.5")
    ap.add_argument("--eps-max", default="40,100,200,700")
    args = ap.parse_args()
    import torch

    vid, cid = codes.dvbs2_like_half()
    dec = qamr.Decoder(vid, cid)
    orc = O.OracleCode(vid, cid)
    ncores = min(len(os.sched_getaffinity(0)), 16)
    for pt in args.points.split(","):
        bps, snr = pt.split(":")
        bps, snr = int(bps), float(snr)
        pipe = SofteningPipeline(dec, bps=bps, snr_db=snr, batch=args.frames)
        g = torch.Generator(device="cuda")
        g.manual_seed(1234 + bps)
        b = pipe.generate(g)
        L = pipe.demap(b)
        torch.cuda.synchronize()
        llr = L[:, :b.B].T.contiguous().cpu().numpy()
        synd = b.synd[:, :b.B].T.contiguous().cpu().numpy()
        s2, i2, f2 = orc.decode_batch(llr, synd, 50, nthreads=ncores)
        fin = np.isfinite(f2)
        print(f"== bps={bps} snr={snr}: frames {b.B}, success {int(s2.sum())}, mean iters {i2.mean():.1f}, "
              f"|lappr| p50/p99/max {np.percentile(np.abs(llr), 50):.1f}/{np.percentile(np.abs(llr), 99):.1f}/"
              f"{np.abs(llr).max():.1f}, |final| p50/p99 {np.percentile(np.abs(f2[fin]), 50):.1f}/"
              f"{np.percentile(np.abs(f2[fin]), 99):.1f}", flush=True)
        runs = [(0, 40), (1, 40)] + [(2, int(e)) for e in args.eps_max.split(",")]
        for eps, emax in runs:
            _lib.tune_set("math", eps)
            _lib.tune_set("eps_max", emax)
            s1, i1, f1 = dec.decode_batch(llr, synd, 50)
            m = np.isfinite(f2) & np.isfinite(f1)
            ratio = np.abs(f1[m] - f2[m]) / (1e-6 * np.abs(f2[m]) + 1e-9)
            print(f"  math={eps} eps_max={emax:4d}: success eq {np.array_equal(s1, s2)}, iters eq "
                  f"{np.array_equal(i1, i2)}, hard eq {np.array_equal(f1 < 0, f2 < 0)}, nan eq "
                  f"{np.array_equal(np.isnan(f1), np.isnan(f2))}, worst err/tol {ratio.max():.3g}, "
                  f"n over tol {(ratio > 1).sum()}, bit-identical share {(f1[m] == f2[m]).mean():.4f}", flush=True)
        _lib.tune_set("math", 0)
        _lib.tune_set("eps_max", 40)


if __name__ == "__main__":
    main()
