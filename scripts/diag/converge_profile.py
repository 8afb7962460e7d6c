#!/usr/bin/env python3
"""Per-launch cost of a converging decode: run it under a kernel trace, then price every degree-7
check launch per running frame.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/conv -o run -- \
        python3 scripts/diag/converge_profile.py --snr 4.0 --out gpurun_out/conv_its.npy
    python3 scripts/diag/converge_profile.py --analyze gpurun_out/conv/run_kernel_trace.csv \
        --its gpurun_out/conv_its.npy

The run decodes the bench's batch (warmup + `--steps` decodes, same inputs every time) and saves
the frames' iteration counts.  The analysis takes the last decode of the trace, pairs its check
launches with (half, iteration) in schedule order (run_split2: C_A(1), C_B(1), C_A(2), ...) and
counts the frames that sweep works on (its >= t - 1: sweep t finds the frames whose posterior
t - 1 satisfies the syndrome), so each launch's
microseconds per running frame can be set against the dense launch's (4.1 ms / 2 048 frames)."""
import argparse
import csv
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)


def run(args):
    import bench

    w = bench.Work("dvbs2_4pam" if args.bps == 2 else "dvbs2_16pam", args.snr, args.batch, 50, 1.0, 0, 0, 0)
    for _ in range(args.steps + 1):
        w.step()
    w.sync()
    np.save(args.out, w.its.cpu().numpy())
    print("mean iterations", w.mean_iterations())


def analyze(args):
    its = np.load(args.its)
    B = its.size
    h = B // 2
    rows = list(csv.DictReader(open(args.analyze)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_init_status" in r["Kernel_Name"]]
    dec = rows[starts[-1]:]
    # the main-loop sweeps only (kFirst / kNormal): the parity-only sweeps (mode 2) of the inputs
    # and of the last posteriors are not part of the pairing
    chk = [r for r in dec if "k_check<7, 0" in r["Kernel_Name"] or "k_check<7, 1" in r["Kernel_Name"]]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    dense = 4100.0 / h
    tot = ideal = 0.0
    out = []
    for k, r in enumerate(chk):
        t, half = k // 2 + 1, k % 2
        # sweep t works on the frames not yet found satisfied: iterations >= t - 1
        run_ = int((its[half * h:(half + 1) * h] >= t - 1).sum())
        d = dur(r)
        tot += d
        ideal += run_ * dense
        out.append((t, "AB"[half], run_, d, d / max(run_, 1)))
    print(f"{len(chk)} check launches, {tot / 1e3:.1f} ms; at the dense cost per running frame "
          f"({dense:.2f} us) {ideal / 1e3:.1f} ms; excess {(tot - ideal) / 1e3:.1f} ms")
    bands = {}
    for t, hf, n, d, per in out:
        key = ("dense >= 90 %" if n >= 0.9 * h else "50-90 %" if n >= 0.5 * h else "10-50 %" if n >= 0.1 * h
               else "65-10 %" if n > 64 else "<= 64")
        b = bands.setdefault(key, [0, 0.0, 0.0])
        b[0] += 1
        b[1] += d
        b[2] += n * dense
    for k, (c, d, i) in bands.items():
        print(f"  running {k:>13}: {c:3d} launches, {d / 1e3:7.2f} ms, ideal {i / 1e3:7.2f} ms, excess {(d - i) / 1e3:6.2f} ms")
    if args.verbose:
        for t, hf, n, d, per in out:
            print(f"  t={t:2d} {hf} running {n:5d}  {d:8.1f} us  {per:6.2f} us/frame")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--snr", type=float, default=4.0)
    ap.add_argument("--bps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/conv_its.npy")
    ap.add_argument("--analyze", default=None)
    ap.add_argument("--its", default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args()
    analyze(args) if args.analyze else run(args)


if __name__ == "__main__":
    main()
