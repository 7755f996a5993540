# round 4: LDS-DMA phase A in the bf16 window kernel -- tests, then alternating A/B (SVOC_WIN_DMA=0/1;
# c3 bf16 also with 4-wave workgroups, SVOC_WIN_W4=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_win_gpu.py tests/test_win_gpu_extra.py tests/test_ops_gpu.py tests/test_revert_gpu.py tests/test_fast_transactional.py tests/test_pipeline_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4_windma_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_windma_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag env... -- bench args
  local tag=$1; shift
  timeout -k 10 200 env "$@" > gpurun_out/r4_windma_$tag.log 2>&1 || { tail -5 gpurun_out/r4_windma_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_windma_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']), round(d['ms_per_step'],4))"
}
for rep in 1 2; do
  run c2_dma0_$rep SVOC_WIN_DMA=0 python bench.py --config c2 --steps 30 --warmup 3
  run c2_dma1_$rep SVOC_WIN_DMA=1 python bench.py --config c2 --steps 30 --warmup 3
  run c3b_dma0_$rep SVOC_WIN_DMA=0 python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
  run c3b_dma1_$rep SVOC_WIN_DMA=1 python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
  run c3b_dma1w4_$rep SVOC_WIN_DMA=1 SVOC_WIN_W4=1 python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
done
