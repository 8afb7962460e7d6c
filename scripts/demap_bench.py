#!/usr/bin/env python3
"""A/B the demapper's root search on the GPU (fast replay vs brute force):
time per batch and bit-identity of the LAPPRs.   python scripts/demap_bench.py [--batch 4096]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qam-reconciliation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    import torch
    import qamr
    from qamr import _lib, codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.dvbs2_like_half()
    dec = qamr.Decoder(vid, cid)
    for bps, snr in ((2, 3.0), (2, 9.5), (4, 13.0), (4, 25.0)):
        pipe = SofteningPipeline(dec, bps, snr, batch=args.batch, max_iterations=1)
        b = pipe.generate(torch.Generator(device="cuda").manual_seed(0))
        res = {}
        for fast in (1, 0, 1):
            _lib.tune_set("demap_fast", fast)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = pipe.demap(b)
            e1.record()
            torch.cuda.synchronize()
            res[fast] = (e0.elapsed_time(e1), out)
        same = torch.equal(res[0][1].view(torch.int64), res[1][1].view(torch.int64))
        print(f"bps={bps} snr={snr:5.1f} B={b.B}: fast {res[1][0]:8.1f} ms  brute {res[0][0]:8.1f} ms  "
              f"speedup {res[0][0] / res[1][0]:5.2f}x  bit-identical={same}", flush=True)
        del pipe, b, res
        torch.cuda.empty_cache()
    _lib.tune_set("demap_fast", 1)


if __name__ == "__main__":
    main()
