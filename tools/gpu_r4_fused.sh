# round 4: fused transactional streaming (window kernel reads updated rows from the batch + commit kernel)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fast_transactional.py tests/test_f32_gpu.py tests/test_pipeline_gpu.py tests/test_revert_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_fused_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r4_fused_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for t in 1 0; do
    timeout -k 10 300 python bench.py --transactional $t --storage fp32 > gpurun_out/r4_fused_$t.log 2>&1 || { tail -5 gpurun_out/r4_fused_$t.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4_fused_$t.log').read().splitlines()[-1]); c=d['config']; print('txn=$t', round(d['value']), round(d['ms_per_step'],3), c.get('pruned_net_fallback_rate'), c.get('ok_fraction'))"
  done
done
