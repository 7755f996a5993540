set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gputest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/r4_gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 && echo smoke ok &&
timeout -k 10 300 python bench.py > gpurun_out/r4_bench_default.log 2>&1 && tail -1 gpurun_out/r4_bench_default.log
