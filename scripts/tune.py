#!/usr/bin/env python3
"""Sweep libqamr's kernel-geometry knobs in ONE process (interleaved rounds) on
the headline workload and print per-kernel times (hipEvent, launch stream).

    python scripts/tune.py [--batch 4096] [--iters 6] [--rounds 3]
"""
import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--grid", default="split=1,2;check_per=2,4,8;nt=0,1")
    ap.add_argument("--var-grid", default="split=2;var_per=2,4,8;check_ft=128,256")
    args = ap.parse_args()
    import torch
    import qamr
    from qamr import _lib, codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.dvbs2_like_half()
    dec = qamr.Decoder(vid, cid)
    pipe = SofteningPipeline(dec, 2, 3.0, batch=args.batch, max_iterations=args.iters)
    gen = torch.Generator(device="cuda").manual_seed(0)
    b = pipe.generate(gen)
    lap = pipe.demap(b)
    fin = torch.empty_like(lap)
    su = torch.empty(b.B, dtype=torch.uint8, device=lap.device)
    it = torch.empty(b.B, dtype=torch.int32, device=lap.device)
    torch.cuda.synchronize()

    def parse(grid):
        keys, vals = [], []
        for part in grid.split(";"):
            k, v = part.split("=")
            keys.append(k)
            vals.append([int(x) for x in v.split(",")])
        return [dict(zip(keys, c)) for c in itertools.product(*vals)]

    ref = None
    results = {}
    configs = parse(args.grid)
    vconfigs = parse(args.var_grid)
    for r in range(args.rounds):
        for cfg in configs + vconfigs:
            for k, v in cfg.items():
                _lib.tune_set(k, v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pipe.decode(lap, b, fin, su, it)
            e1.record()
            torch.cuda.synchronize()
            wall = e0.elapsed_time(e1)
            qamr.profile_reset()
            qamr.profile_enable(True)
            pipe.decode(lap, b, fin, su, it)
            torch.cuda.synchronize()
            qamr.profile_enable(False)
            key = json.dumps(cfg, sort_keys=True)
            rec = results.setdefault(key, {"check_d7": [], "var": [], "wall": [], "fused": []})
            rec["wall"].append(wall / args.iters)
            ms, n = qamr.profile_query("fused_d7")
            rec["fused"].append(ms / max(n, 1))
            ms, n = qamr.profile_query("check_d7")
            rec["check_d7"].append(ms / max(n, 1))
            ms, n = qamr.profile_query("var")
            rec["var"].append(ms / max(n, 1))
            # results must not depend on geometry
            h = (int(su.sum()), int(it.sum()), float(fin[:, : b.B].double().abs().sum()))
            if ref is None:
                ref = h
            elif h != ref:
                print("MISMATCH", cfg, h, ref, flush=True)
            for k in cfg:
                _lib.tune_set(k, {"check_ft": 256, "check_per": 4, "var_ft": 256, "var_per": 4, "nt": 1,
                                  "split": 2}[k])
    rows = []
    for key, rec in results.items():
        rows.append((min(rec["wall"]), min(rec["check_d7"]), min(rec["var"]), min(rec["fused"]), key))
    rows.sort()
    print(f"{'ms/iter':>8} {'check_d7':>9} {'var':>7} {'fused_d7':>9}  config   (kernel columns: ms per launch)")
    for w, c, v, fu, k in rows:
        print(f"{w:8.3f} {c:9.3f} {v:7.3f} {fu:9.3f}  {k}")


if __name__ == "__main__":
    main()
