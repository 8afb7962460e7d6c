#!/usr/bin/env python3
"""configs[1] (reg-(3,6) N=1008, 4-PAM 3 dB, B = 1024, 50 iterations): decode time per batch
with the frame-resident decode (resident = 1), the one-launch-per-iteration schedule
(fused_iter = 1) and the flat three-launch schedule (fused_iter = 0), and bit-identity of the outputs.   python scripts/small_ab.py [--reps 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qam-reconciliation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--knobs", default="resident=1;resident=0,fused_iter=1,iter_streams=2;"
                    "resident=0,fused_iter=1,iter_streams=1;resident=0,fused_iter=0")
    args = ap.parse_args()
    import torch
    import qamr
    from qamr import _lib, codes
    from qamr.pipeline import SofteningPipeline

    vid, cid = codes.regular_code(1008)
    dec = qamr.Decoder(vid, cid)
    pipe = SofteningPipeline(dec, 2, 3.0, batch=args.batch, max_iterations=50)
    b = pipe.generate(torch.Generator(device="cuda").manual_seed(0))
    lap = pipe.demap(b)
    res, outs = {}, {}
    for spec in args.knobs.split(";"):
        kv = dict(x.split("=") for x in spec.split(",") if x)
        saved = {k: _lib.tune_get(k) for k in kv}
        for k, v in kv.items():
            _lib.tune_set(k, int(v))
        o = pipe.decode(lap, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            pipe.decode(lap, b, *o)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        res[spec] = {"ms_per_batch": round(ms, 4), "frames_per_s": round(b.B / ms * 1e3, 1),
                     "us_per_iteration": round(1e3 * ms / max(1e-9, float(o[2].float().mean())), 2)}
        outs[spec] = [x.clone() for x in o]
        for k, v in saved.items():
            _lib.tune_set(k, v)
    ref = list(outs.values())[0]
    same = all(torch.equal(o[0][:, :b.B].view(torch.int64), ref[0][:, :b.B].view(torch.int64)) and
               torch.equal(o[1], ref[1]) and torch.equal(o[2], ref[2]) for o in outs.values())
    print(json.dumps({"configs1": res, "bit_identical": same, "mean_iterations": float(ref[2].float().mean())}))
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
