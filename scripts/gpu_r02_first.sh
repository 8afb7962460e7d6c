set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02_gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err
