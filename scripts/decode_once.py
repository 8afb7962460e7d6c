#!/usr/bin/env python3
"""One batched decode of the headline workload (for rocprofv3 --pmc passes):
    QAMR_TUNE=split=1,nt=1 python scripts/decode_once.py [--batch 4096] [--iters 3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qam-reconciliation_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--iters", type=int, default=3)
args = ap.parse_args()
import torch  # noqa: E402
import qamr  # noqa: E402
from qamr import codes  # noqa: E402
from qamr.pipeline import SofteningPipeline  # noqa: E402

vid, cid = codes.dvbs2_like_half()
dec = qamr.Decoder(vid, cid)
pipe = SofteningPipeline(dec, 2, 3.0, batch=args.batch, max_iterations=args.iters)
b = pipe.generate(torch.Generator(device="cuda").manual_seed(0))
lap = pipe.demap(b)
fin, su, it = pipe.decode(lap, b)
torch.cuda.synchronize()
print("decoded", int(su.sum()), float(it.float().mean()))
