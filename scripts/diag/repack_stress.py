#!/usr/bin/env python3
"""Stress the column repack: many seeded B = 4096 converging batches, every frame's outputs
(final LAPPRs as bits, success, iterations) compared between the default decode (repack with
transitions, repack_pct 80) and the decode without the repack and with repack_pct 50.

    python scripts/diag/repack_stress.py [--seeds 8] [--snrs 2:3.8,2:4.0,2:4.2,4:14.0,4:14.5,4:15.0]

Prints one line per batch (repacks per range, final widths, mean iterations, equal or not) and
exits non-zero on the first difference."""
import argparse
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--snrs", default="2:3.8,2:4.0,2:4.2,4:14.0,4:14.5,4:15.0")
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    import torch
    import qamr
    from qamr import _lib, codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.dvbs2_like_half()
    dec = qamr.Decoder(vid, cid)
    names = ("repack", "repack_pct")
    saved = {k: _lib.tune_get(k) for k in names}
    bad = 0
    try:
        for spec in args.snrs.split(","):
            bps, snr = int(spec.split(":")[0]), float(spec.split(":")[1])
            pipe = SofteningPipeline(dec, bps=bps, snr_db=snr, batch=args.batch, max_iterations=50)
            for seed in range(args.seeds):
                b = pipe.generate(torch.Generator(device="cuda").manual_seed(1000 + seed))
                lappr = pipe.demap(b)
                outs, stats = [], []
                for t in (dict(), dict(repack=0), dict(repack_pct=50)):
                    for k, v in saved.items():
                        _lib.tune_set(k, t.get(k, v))
                    outs.append([x.clone() for x in pipe.decode(lappr, b)])
                    torch.cuda.synchronize()
                    stats.append(dec.repack_stats(pipe.ld, 50))
                f0, s0, i0 = outs[0]
                same = all(torch.equal(s0, s) and torch.equal(i0, i) and
                           torch.equal(f0[:, :args.batch].view(torch.int64), f[:, :args.batch].view(torch.int64))
                           for f, s, i in outs[1:])
                print(f"bps={bps} {snr} dB seed {seed}: repacks {stats[0][0]} widths {stats[0][1]} "
                      f"(pct 50: {stats[2][0]}), mean iterations {float(i0.float().mean()):.2f}, "
                      f"successes {int(s0.sum())}, {'identical' if same else 'DIFFERENT'}", flush=True)
                if not same:
                    bad += 1
                    return 1
    finally:
        for k, v in saved.items():
            _lib.tune_set(k, v)
    print(f"all identical ({bad} differences)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
