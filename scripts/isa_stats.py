#!/usr/bin/env python3
"""Per-kernel static ISA statistics of a gfx950 device assembly file (hipcc --cuda-device-only -S):
VGPRs, AGPRs, SGPRs, scratch bytes, static instruction count and the count per opcode class.

  python scripts/isa_stats.py decoder.s [--filter k_check] [--opcodes]

Used to check that a refactor leaves a hot kernel's code unchanged (same register budget and
instruction mix) before spending GPU time on it."""
import argparse
import collections
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return dict(zip(names, out))
    except Exception:
        return {n: n for n in names}


def parse(path):
    kernels = {}
    cur = None
    meta = None
    for line in open(path):
        s = line.strip()
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and not line.startswith(" ") and not line.startswith("\t"):
            cur = m.group(1)
            kernels.setdefault(cur, {"insts": 0, "ops": collections.Counter()})
            continue
        if cur and s.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur and re.match(r"^(s_|v_|ds_|buffer_|global_|flat_|scratch_)", s):
            kernels[cur]["insts"] += 1
            kernels[cur]["ops"][s.split()[0]] += 1
            continue
        m = re.match(r"^\.amdhsa_kernel\s+(\S+)", s)
        if m:
            meta = m.group(1)
            kernels.setdefault(meta, {"insts": 0, "ops": collections.Counter()})
            continue
        if meta:
            for key, tag in ((".amdhsa_next_free_vgpr", "vgpr"), (".amdhsa_next_free_sgpr", "sgpr"),
                             (".amdhsa_private_segment_fixed_size", "scratch"),
                             (".amdhsa_accum_offset", "accum_offset"),
                             (".amdhsa_group_segment_fixed_size", "lds")):
                if s.startswith(key + " "):
                    kernels[meta][tag] = int(s.split()[1], 0)
            if s.startswith(".end_amdhsa_kernel"):
                meta = None
    return kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--filter", default="")
    ap.add_argument("--opcodes", action="store_true")
    a = ap.parse_args()
    ks = parse(a.asm)
    dm = demangle(list(ks))
    for k in sorted(ks, key=lambda n: dm[n]):
        name = dm[k]
        if a.filter and a.filter not in name:
            continue
        d = ks[k]
        if "vgpr" not in d:
            continue
        print(f"{name}: vgpr={d.get('vgpr')} (arch {d.get('accum_offset', '?')}) sgpr={d.get('sgpr')} "
              f"scratch={d.get('scratch')} lds={d.get('lds')} insts={d['insts']}")
        if a.opcodes:
            for op, n in sorted(d["ops"].items()):
                print(f"    {op} {n}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
