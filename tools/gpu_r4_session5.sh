# round 4: bf16 window kernel without implicit fp contraction -- tests + c3 bf16 / c2 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fast_transactional.py tests/test_win_gpu.py tests/test_win_gpu_extra.py tests/test_ops_gpu.py tests/test_revert_gpu.py tests/test_pipeline_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_s5_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_s5_tests.log; [ $rc -eq 0 ] || exit $rc
for a in "c3 --storage bf16" "c2" "c3 --storage bf16 --transactional 0"; do
  timeout -k 10 300 python bench.py --config $a --steps 20 --warmup 3 > gpurun_out/r4_s5.log 2>&1 || { tail -3 gpurun_out/r4_s5.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_s5.log').read().strip().splitlines()[-1]); print('$a', round(d['value']), round(d['ms_per_step'],3))"
done
