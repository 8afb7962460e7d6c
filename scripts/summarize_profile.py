#!/usr/bin/env python3
"""Summarise a scripts/profile_session.sh output directory.

    python scripts/summarize_profile.py gpurun_out/prof_r1 [--kernel 'k_check<7, 1, true>'] [--kernel-key check_d7]
        [--workload dvbs2_4pam --batch 4096] [--source TEXT] [--into profiles/pmc_secondary.json]

Writes <dir>/summary.md (per-kernel time from --kernel-trace --stats, PMC counters
per launch) and <dir>/pmc_traffic.json: HBM bytes per launch of the dominant
kernel = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 -- the gfx950 corrections of
MI355X_MICROARCH.md 'HBM': FETCH_SIZE (KiB) counts half the bytes of wide
coalesced reads (calibrated here on the variable sweep, whose read bytes are
known exactly), WRITE_SIZE (KiB) is exact.  --into merges the record into a JSON list of such
records (one per workload, batch and kernel key: bench.py's pmc_entry reads them).
"""
import argparse
import collections
import csv
import glob
import json
import os


def short(name):
    return name.split("(")[0].replace("void ", "").replace("qr::", "").strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_check<7, 1, true>")
    ap.add_argument("--kernel-key", default="check_d7")
    ap.add_argument("--source", default=None, help="provenance text stored in the record")
    ap.add_argument("--into", default=None, help="JSON list of records to merge this one into")
    ap.add_argument("--workload", default="dvbs2_4pam")
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    d = args.dir
    lines = []
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    avg_ns = {}
    if os.path.exists(stats):
        lines.append("| kernel | calls | avg us | total ms | % |\n|---|---|---|---|---|")
        for r in csv.DictReader(open(stats)):
            k = short(r["Name"])
            avg_ns[k] = float(r["AverageNs"])
            lines.append(f"| `{k}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                         f"{float(r['TotalDurationNs']) / 1e6:.1f} | {float(r['Percentage']):.1f} |")
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if ctr:
        names = sorted({c for k in ctr.values() for c in k})
        lines.append("\n| kernel | " + " | ".join(names) + " |\n|---|" + "---|" * len(names))
        for k, cs in sorted(ctr.items(), key=lambda kv: -max((sum(v) / len(v) for v in kv[1].values()), default=0)):
            if not any(x in k for x in ("k_fused", "k_check", "k_var", "k_demap", "k_bob", "k_resident", "k_iter")):
                continue
            vals = [f"{sum(cs[n]) / len(cs[n]):.4g}" if cs.get(n) else "" for n in names]
            lines.append(f"| `{k}` | " + " | ".join(vals) + " |")
    out = {}
    kc = ctr.get(args.kernel, {})
    if kc.get("FETCH_SIZE") and kc.get("WRITE_SIZE"):
        fetch = sum(kc["FETCH_SIZE"]) / len(kc["FETCH_SIZE"])
        write = sum(kc["WRITE_SIZE"]) / len(kc["WRITE_SIZE"])
        out = {"workload": args.workload, "batch": args.batch, "kernel": args.kernel, "kernel_key": args.kernel_key,
               "fetch_size_kib": fetch, "write_size_kib": write,
               "hbm_bytes_per_launch": int((2 * fetch + write) * 1024),
               "correction": "2*FETCH_SIZE + WRITE_SIZE, KiB -> bytes (MI355X_MICROARCH.md HBM section)",
               "avg_launch_us_trace": avg_ns.get(args.kernel, 0) / 1e3}
        avg = lambda n: sum(kc[n]) / len(kc[n]) if kc.get(n) else None  # noqa: E731
        if avg("SQ_INSTS_VALU"):
            out["valu_insts_per_launch"] = avg("SQ_INSTS_VALU")
            f64 = [avg(n) for n in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                    "SQ_INSTS_VALU_TRANS_F64") if avg(n) is not None]
            if f64:
                out["valu_f64_insts_per_launch"] = sum(f64)
        # VALUBusy as rocprofv3 defines it: SQ_ACTIVE_INST_VALU (quad-cycles, summed over the
        # SIMDs) / CU_NUM / GRBM_GUI_ACTIVE (per XCD); every wave64 VALU instruction -- fp64
        # or 32-bit -- occupies one quad-cycle of its SIMD here.  The shader clock during the
        # launch = GRBM_GUI_ACTIVE per XCD / the traced launch time.
        xcds, cus = 8, 256
        if avg("SQ_ACTIVE_INST_VALU") and avg("GRBM_GUI_ACTIVE"):
            grbm_xcd = avg("GRBM_GUI_ACTIVE") / xcds
            out["valu_busy_pmc"] = avg("SQ_ACTIVE_INST_VALU") / cus / grbm_xcd
            if avg_ns.get(args.kernel):
                out["clock_ghz_pmc"] = grbm_xcd / avg_ns[args.kernel]
        if args.source:
            out["source"] = args.source
        json.dump(out, open(os.path.join(d, "pmc_traffic.json"), "w"), indent=1)
        if args.into:
            try:
                recs = json.load(open(args.into))
            except Exception:
                recs = []
            recs = [r for r in recs if (r.get("workload"), r.get("batch"), r.get("kernel_key"))
                    != (out["workload"], out["batch"], out["kernel_key"])] + [out]
            json.dump(recs, open(args.into, "w"), indent=1)
        lines.append(f"\nDominant kernel `{args.kernel}`: HBM traffic per launch "
                     f"{out['hbm_bytes_per_launch'] / 1e9:.2f} GB (2*FETCH + WRITE)")
    open(os.path.join(d, "summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
