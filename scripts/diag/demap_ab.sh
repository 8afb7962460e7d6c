# Demap cost breakdown: default vs no LLR sums vs no root search (timing only; the variants are wrong on purpose).
for L in qam-reconciliation_amd/qamr/libqamr.so qam-reconciliation_amd/qamr/exp/libqamr_nollr.so qam-reconciliation_amd/qamr/exp/libqamr_nosearch.so; do
  echo "== $L"; QAMR_LIB=$L timeout -k 10 200 python scripts/demap_bench.py 2>&1 | grep -v amdgpu.ids | tail -8
done
