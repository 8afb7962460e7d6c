set -o pipefail
timeout -k 10 400 python -u scripts/diag/eps_accuracy.py --eps-max 40,700 > gpurun_out/eps_acc.txt 2>&1
L="qam-reconciliation_amd/qamr/libqamr.so qam-reconciliation_amd/qamr/exp/libqamr_sw4.so qam-reconciliation_amd/qamr/exp/libqamr_sw6.so"
LIBS="$L" TUNES="math=0" STEPS=3 bash scripts/exp_bench.sh > gpurun_out/ab_strict.txt 2>&1
LIBS="qam-reconciliation_amd/qamr/libqamr.so" TUNES="math=1;math=2" STEPS=3 bash scripts/exp_bench.sh >> gpurun_out/ab_strict.txt 2>&1
