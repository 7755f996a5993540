# round 4: c5 step (small kernel commits c1, short-row update with one round trip, restore grid)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_revert_gpu.py tests/test_fast_transactional.py tests/test_pipeline_gpu.py tests/test_legacy.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4_c5_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_c5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 --steps 200 --warmup 20 > gpurun_out/r4_c5_bench.log 2>&1 || { tail -5 gpurun_out/r4_c5_bench.log; exit 1; }
tail -1 gpurun_out/r4_c5_bench.log | cut -c1-220
CFGS=c5:20 ANCHOR=consensus bash tools/prof_steps.sh
