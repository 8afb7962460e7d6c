#!/usr/bin/env python3
"""Diagnostic: do the decode's per-launch hipEvent pairs survive HIP-graph capture?
Captures a profiled decode (N=64800, B=512) and reports the kernel stats after replays,
beside an eager profiled decode and the wall time per decode of both."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "qam-reconciliation_amd"))
import torch  # noqa: E402
import qamr  # noqa: E402
from qamr import codes  # noqa: E402
from qamr.pipeline import SofteningPipeline  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
vid, cid = codes.dvbs2_like_half()
dec = qamr.Decoder(vid, cid)
pipe = SofteningPipeline(dec, 2, 3.0, batch=B)
b = pipe.generate(torch.Generator(device="cuda").manual_seed(0))
L = pipe.demap(b)
fin, succ, its = pipe.decode(L, b)
torch.cuda.synchronize()


def stats(tag):
    out = {}
    for k in ("check_d7", "var", "status"):
        ms, n = qamr.profile_query(k)
        out[k] = (round(1e3 * ms / n, 1) if n else None, n)
    print(tag, out, flush=True)


for eager in (True, False):
    qamr.profile_reset()
    qamr.profile_enable(True)
    if eager:
        t0 = time.perf_counter()
        pipe.decode(L, b, fin, succ, its)
        torch.cuda.synchronize()
        qamr.profile_enable(False)
        print("eager wall ms", round(1e3 * (time.perf_counter() - t0), 2))
        stats("eager")
    else:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            pipe.decode(L, b, fin, succ, its)
        qamr.profile_enable(False)
        print("last error after capture:", qamr._lib.load().qr_last_error().decode()[:200])
        for _ in range(2):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        print("graph wall ms per decode", round(1e3 * (time.perf_counter() - t0) / 5, 2))
        stats("graph")
