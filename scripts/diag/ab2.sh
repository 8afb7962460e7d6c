set -o pipefail
timeout -k 10 400 python -u scripts/diag/eps_accuracy.py > gpurun_out/eps_acc.txt 2>&1 && \
LIBS="qam-reconciliation_amd/qamr/libqamr.so" TUNES="eps_max=100;eps_max=200;eps_max=700" STEPS=2 BENCH_ARGS="--workload dvbs2_16pam" bash scripts/exp_bench.sh > gpurun_out/ab_16pam_emax.txt 2>&1
