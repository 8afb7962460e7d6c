#!/bin/bash
# Demap-only experiment variant: recompile demap.hip with FLAGS, link with the default
# build's decoder.o / runtime.o:  scripts/exp_build_demap.sh NAME "-DFLAG ..."
# -> qam-reconciliation_amd/qamr/exp/libqamr_NAME.so (QAMR_LIB=... selects it)
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2
out=qam-reconciliation_amd/qamr/exp
b=qam-reconciliation_amd/csrc/build
mkdir -p $out /tmp/qamr_exp_$name
make -s -C qam-reconciliation_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fvisibility=hidden -Iinclude -I$b $flags -c qam-reconciliation_amd/csrc/demap.hip -o /tmp/qamr_exp_$name/demap.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libqamr_$name.so $b/runtime.o $b/decoder.o /tmp/qamr_exp_$name/demap.o
echo $out/libqamr_$name.so
