#!/bin/bash
# Demap timing over library variants: LIBS="a.so b.so" bash scripts/demap_cmp.sh
for L in ${LIBS:-qam-reconciliation_amd/qamr/libqamr.so}; do echo $L; QAMR_LIB=$L timeout -k 10 300 python scripts/demap_bench.py 2>&1 | grep bps= || exit 1; done
