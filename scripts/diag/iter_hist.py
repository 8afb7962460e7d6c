"""Diagnostic: iteration-count histogram of the bench batch at an operating point (how many
frames are still running at each iteration), to price the converging schedule's launches.
   python scripts/diag/iter_hist.py [--workload dvbs2_4pam] [--snr 4.0] [--batch 4096]"""
import argparse
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="dvbs2_4pam")
    ap.add_argument("--snr", type=float, default=4.0)
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    import numpy as np
    import bench

    w = bench.Work(args.workload, args.snr, args.batch, 50, 1.0, 0, 0, 0)
    w.step()
    w.sync()
    its = w.its.cpu().numpy()
    succ = w.succ.cpu().numpy()
    h = np.bincount(its, minlength=51)
    B = len(its)
    # frames still running in iteration t's check sweep (t = 1..50): those with iters >= t, plus
    # failures (iters = 50, success 0)
    running = [int(((its >= t) & ~((its == t - 1) & (succ == 1))).sum()) for t in range(1, 51)]
    half = B // 2
    run_a = [int(((its[:half] >= t)).sum()) for t in range(1, 51)]
    run_b = [int(((its[half:] >= t)).sum()) for t in range(1, 51)]
    print(json.dumps({"workload": args.workload, "snr": args.snr, "B": B, "mean_iterations": float(its.mean()),
                      "failures": int((succ == 0).sum()), "hist": h.tolist(), "running": running,
                      "running_half_a": run_a, "running_half_b": run_b}))


if __name__ == "__main__":
    main()
