#!/bin/bash
# Build an experiment variant of libqamr.so: scripts/exp_build.sh NAME "-DFLAG ..."
# -> qam-reconciliation_amd/qamr/exp/libqamr_NAME.so (load with QAMR_LIB=...).
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2
out=qam-reconciliation_amd/qamr/exp
mkdir -p $out /tmp/qamr_exp_$name
make -s -C qam-reconciliation_amd/csrc "$PWD/qam-reconciliation_amd/csrc/build/glibc_tables.inc"
for s in runtime decoder demap; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
    -fvisibility=hidden -Iinclude -Iqam-reconciliation_amd/csrc/build $flags -c qam-reconciliation_amd/csrc/$s.hip -o /tmp/qamr_exp_$name/$s.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libqamr_$name.so /tmp/qamr_exp_$name/*.o
echo $out/libqamr_$name.so
