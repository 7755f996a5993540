# round 4: transactional fast streaming (tests + c3 overhead A/B) and the phase-A DMA stream rate
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/dma_rate > gpurun_out/r4_dma_rate.txt 2>&1; cat gpurun_out/r4_dma_rate.txt
timeout -k 10 600 python -u -m pytest tests/test_fast_transactional.py tests/test_revert_gpu.py tests/test_pipeline_gpu.py tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_txn_tests.log 2>&1 && tail -2 gpurun_out/r4_txn_tests.log &&
for r in 1 2; do
  for t in 1 0; do
    timeout -k 10 300 python bench.py --transactional $t --storage fp32 > gpurun_out/r4_txn_ab_$t.log 2>&1 && python -c "import json,sys; d=json.loads(open('gpurun_out/r4_txn_ab_$t.log').read().splitlines()[-1]); print('txn=$t', round(d['value']), d['ms_per_step'], d['config'].get('fast_transactional'))" || exit 1
  done
done
