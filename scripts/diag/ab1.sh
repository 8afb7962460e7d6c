set -o pipefail
L="qam-reconciliation_amd/qamr/libqamr.so qam-reconciliation_amd/qamr/exp/libqamr_listfb.so qam-reconciliation_amd/qamr/exp/libqamr_w4.so"
LIBS="$L" TUNES="eps=1;eps=0" STEPS=3 bash scripts/exp_bench.sh > gpurun_out/ab_4pam.txt 2>&1 && \
LIBS="qam-reconciliation_amd/qamr/libqamr.so qam-reconciliation_amd/qamr/exp/libqamr_w4.so" TUNES="eps=1;eps=0" STEPS=2 BENCH_ARGS="--workload dvbs2_16pam" bash scripts/exp_bench.sh > gpurun_out/ab_16pam.txt 2>&1
