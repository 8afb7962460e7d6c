#!/bin/bash
# Device assembly of decoder.hip with the library's flags (for scripts/isa_stats.py):
#   bash scripts/dev_asm.sh out.s [EXTRA_FLAGS...]
set -eu
R="$(cd "$(dirname "$0")/.." && pwd)"
C="$R/qam-reconciliation_amd/csrc"
out=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
    -I"$R/include" -I"$C/build" --cuda-device-only -S "$@" -o "$out" "$C/decoder.hip"
