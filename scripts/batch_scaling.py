#!/usr/bin/env python3
"""Per-frame kernel cost vs batch size (does a small frame tile stay resident in
the 256 MiB Infinity Cache?).  One process, hipEvent timing on the launch stream."""
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
    iters = int(os.environ.get("ITERS", "8"))
    for nt in (0, 1):
        _lib.tune_set("nt", nt)
        for B in (64, 128, 256, 512, 1024, 2048, 4096):
            pipe = SofteningPipeline(dec, 2, 3.0, batch=B, max_iterations=iters)
            gen = torch.Generator(device="cuda").manual_seed(0)
            b = pipe.generate(gen)
            lap = pipe.demap(b)
            fin = torch.empty_like(lap)
            su = torch.empty(b.B, dtype=torch.uint8, device=lap.device)
            it = torch.empty(b.B, dtype=torch.int32, device=lap.device)
            pipe.decode(lap, b, fin, su, it)  # warm
            torch.cuda.synchronize()
            best = {}
            for _ in range(3):
                qamr.profile_reset()
                qamr.profile_enable(True)
                pipe.decode(lap, b, fin, su, it)
                torch.cuda.synchronize()
                qamr.profile_enable(False)
                for k in ("check_d7", "var", "status"):
                    ms, n = qamr.profile_query(k)
                    v = ms / max(n, 1)
                    best[k] = min(best.get(k, 1e9), v)
            print(f"nt={nt} B={B:5d}  check_d7 {best['check_d7']*1e3:9.1f} us ({best['check_d7']*1e3/B:6.3f} us/frame)"
                  f"  var {best['var']*1e3:8.1f} us ({best['var']*1e3/B:6.3f} us/frame)  status {best['status']*1e3:6.1f} us",
                  flush=True)
            del pipe, b, lap, fin
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
