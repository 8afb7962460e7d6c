#!/usr/bin/env python3
"""A/B of runtime knobs (qr_tune_set) on one resident batch: ms per step and frames/s for each
knob set, interleaved over rounds (so box drift hits every variant alike), outputs compared
bit for bit against the first variant.
    python scripts/knob_ab.py --workload dvbs2_4pam --snr 4.0 --knobs "check_queue=1;check_queue=0"
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="dvbs2_4pam")
    ap.add_argument("--snr", type=float, default=None)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--knobs", required=True, help="variants separated by ';', knobs by ','")
    args = ap.parse_args()
    import torch
    import bench
    from qamr import _lib

    w = bench.Work(args.workload, args.snr, args.batch, 50, 1.0, 0, 0, 0)
    variants = [dict((k, int(v)) for k, v in (x.split("=") for x in spec.split(",") if x))
                for spec in args.knobs.split(";")]
    names = sorted({k for v in variants for k in v})
    saved = {k: _lib.tune_get(k) for k in names}
    times = {i: [] for i in range(len(variants))}
    ref = None
    same = {}
    try:
        for r in range(args.rounds):
            for i, v in enumerate(variants):
                for k in names:
                    _lib.tune_set(k, v.get(k, saved[k]))
                w.step_eager()
                w.sync()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    w.step_eager()
                w.sync()
                times[i].append((time.perf_counter() - t0) / args.steps)
                out = (w.final[:, :w.B].clone(), w.succ.clone(), w.its.clone())
                if ref is None:
                    ref = out
                same[i] = same.get(i, True) and all(torch.equal(a.view(torch.int64) if a.dtype == torch.float64 else a,
                                                                b.view(torch.int64) if b.dtype == torch.float64 else b)
                                                    for a, b in zip(out, ref))
    finally:
        for k, v in saved.items():
            _lib.tune_set(k, v)
    for i, v in enumerate(variants):
        t = min(times[i])
        print(json.dumps({"variant": v, "workload": args.workload, "snr": w.snr, "ms_per_step": round(1e3 * t, 3),
                          "frames_per_s": round(w.B / t, 1), "all_ms": [round(1e3 * x, 2) for x in times[i]],
                          "mean_iterations": round(w.mean_iterations(), 3), "bit_identical": same[i]}), flush=True)
    sys.exit(0 if all(same.values()) else 1)


if __name__ == "__main__":
    main()
