#!/usr/bin/env python3
"""Does a small frame block decoded through all its iterations stay resident in the
256 MiB Infinity Cache, and what does it cost per frame-iteration?  Whole-decode
wall time (torch events) and per-kernel hipEvent times, for small batches and
several check_per / var_per settings."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qam-reconciliation_amd"))


def main():
    import torch
    import qamr
    from qamr import _lib, codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.dvbs2_like_half()
    dec = qamr.Decoder(vid, cid)
    iters = int(os.environ.get("ITERS", "20"))
    Bs = [int(x) for x in os.environ.get("BS", "64,128,256,4096").split(",")]
    pers = [int(x) for x in os.environ.get("PERS", "1,2,4,16").split(",")]
    for B in Bs:
        pipe = SofteningPipeline(dec, 2, 3.0, batch=B, max_iterations=iters)
        gen = torch.Generator(device="cuda").manual_seed(0)
        b = pipe.generate(gen)
        lap = pipe.demap(b)
        fin = torch.empty_like(lap)
        su = torch.empty(b.B, dtype=torch.uint8, device=lap.device)
        it = torch.empty(b.B, dtype=torch.int32, device=lap.device)
        for nt in (0, 1):
            for per in pers:
                for vper in (2, 8):
                    _lib.tune_set("nt", nt)
                    _lib.tune_set("check_per", per)
                    _lib.tune_set("var_per", vper)
                    pipe.decode(lap, b, fin, su, it)  # warm
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    reps = 3
                    e0.record()
                    for _ in range(reps):
                        pipe.decode(lap, b, fin, su, it)
                    e1.record()
                    torch.cuda.synchronize()
                    wall = e0.elapsed_time(e1) / reps
                    qamr.profile_reset()
                    qamr.profile_enable(True)
                    pipe.decode(lap, b, fin, su, it)
                    torch.cuda.synchronize()
                    qamr.profile_enable(False)
                    ks = {}
                    for k in ("check_d7", "fused_d7", "var", "status"):
                        ms, n = qamr.profile_query(k)
                        if n:
                            ks[k] = ms / n * 1e3
                    fi = wall * 1e3 / (B * iters)
                    print(f"B={B:5d} nt={nt} per={per:2d} vper={vper} wall {wall:8.3f} ms = {fi:6.3f} us/frame-it  "
                          + "  ".join(f"{k} {v:8.1f}us" for k, v in ks.items()), flush=True)
        del pipe, b, lap, fin
        torch.cuda.empty_cache()
    _lib.tune_set("nt", 1)


if __name__ == "__main__":
    main()
