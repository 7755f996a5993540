# round 4: pruned window network (fp32 N = 256) + transactional fast streaming: tests, c3 bench, DMA rate
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/dma_rate > gpurun_out/r4_dma_rate.txt 2>&1; cat gpurun_out/r4_dma_rate.txt
timeout -k 10 600 python -u -m pytest tests/test_f32_gpu.py tests/test_fast_transactional.py tests/test_revert_gpu.py tests/test_pipeline_gpu.py tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_prune_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_prune_tests.log; [ $rc -eq 0 ] || exit $rc
for t in 1 0 1; do
  timeout -k 10 300 python bench.py --transactional $t --storage fp32 > gpurun_out/r4_c3_txn$t.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r4_c3_txn$t.log').read().splitlines()[-1]); c=d['config']; print('txn=$t', round(d['value']), round(d['ms_per_step'],3), c.get('fast_transactional'), c.get('pruned_net_fallback_rate'))"
done
