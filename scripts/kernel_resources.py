#!/usr/bin/env python3
"""Register allocation of every kernel in a built HIP library, read from the gfx950 code object
itself (the .hip_fatbin section's clang offload bundle -> the AMDGPU ELF -> its amdhsa metadata
note): name, VGPRs allocated (.vgpr_count), SGPRs, scratch bytes per lane, LDS bytes.

    python scripts/kernel_resources.py [qam-reconciliation_amd/qamr/libqamr.so] [--filter k_repack]

Used by tests/test_vgpr_budget.py (the register note of decoder.hip: kernels launched beside the
check sweep allocate 16 or 32 VGPRs, never 24)."""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB = os.path.join(ROOT, "qam-reconciliation_amd", "qamr", "libqamr.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def section(path, name):
    """(file offset, size) of an ELF64 section by name."""
    with open(path, "rb") as f:
        data = f.read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    stroff = sh(shstrndx)[4]
    for i in range(shnum):
        s = sh(i)
        nm = data[stroff + s[0]:data.index(b"\0", stroff + s[0])].decode()
        if nm == name:
            return data, s[4], s[5]
    raise KeyError(f"{path}: no section {name}")


def code_objects(path, arch="gfx950"):
    """The device ELF images for `arch` inside the library's offload bundles."""
    data, off, size = section(path, ".hip_fatbin")
    blob = data[off:off + size]
    out = []
    pos = 0
    while True:
        b = blob.find(MAGIC, pos)
        if b < 0:
            break
        n, = struct.unpack_from("<Q", blob, b + len(MAGIC))
        p = b + len(MAGIC) + 8
        end = b
        for _ in range(n):
            eoff, esz, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if arch in triple and esz:
                out.append(blob[b + eoff:b + eoff + esz])
            end = max(end, b + eoff + esz)
        pos = max(end, b + len(MAGIC))
    return out


def kernels(path=LIB, arch="gfx950"):
    """{kernel symbol name: {"vgpr", "sgpr", "scratch", "lds", "agpr"}} from the amdhsa notes."""
    import yaml

    res = {}
    for co in code_objects(path, arch):
        with tempfile.NamedTemporaryFile(suffix=".co") as t:
            t.write(co)
            t.flush()
            txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", t.name], capture_output=True,
                                 text=True, check=True).stdout
        i = txt.index("amdhsa.kernels:")
        j = txt.find("\n...", i)
        meta = yaml.safe_load(txt[i:j if j > 0 else None])
        for k in meta["amdhsa.kernels"]:
            res[k[".symbol"]] = {"name": k[".name"], "vgpr": k[".vgpr_count"], "sgpr": k[".sgpr_count"],
                                 "scratch": k[".private_segment_fixed_size"], "lds": k[".group_segment_fixed_size"],
                                 "agpr": k.get(".agpr_count", 0), "vgpr_spill": k.get(".vgpr_spill_count", 0)}
    return res


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return dict(zip(names, out))
    except Exception:
        return {n: n for n in names}


def main():
    args = sys.argv[1:]
    flt = None
    if "--filter" in args:
        i = args.index("--filter")
        flt = args[i + 1]
        del args[i:i + 2]
    path = args[0] if args else LIB
    ks = kernels(path)
    dm = demangle([k.removesuffix(".kd") for k in ks])
    for sym, r in sorted(ks.items(), key=lambda kv: dm.get(kv[0].removesuffix(".kd"), kv[0])):
        name = dm.get(sym.removesuffix(".kd"), sym)
        if flt and flt not in name:
            continue
        print(f"{r['vgpr']:4d} VGPR {r['sgpr']:4d} SGPR {r['scratch']:5d} B scratch {r['lds']:6d} B LDS  {name}")


if __name__ == "__main__":
    main()
