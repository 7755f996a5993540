# round 4: fused transactional streaming in the bf16 window kernel -- tests, then c3 bf16 A/B (fused / generic / none)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fast_transactional.py tests/test_win_gpu.py tests/test_win_gpu_extra.py tests/test_ops_gpu.py tests/test_revert_gpu.py tests/test_pipeline_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_s4_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_s4_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag env... -- bench args
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r4_s4_$tag.log 2>&1 || { tail -5 gpurun_out/r4_s4_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_s4_$tag.log').read().strip().splitlines()[-1]); c=d['config']; print('$tag', round(d['value']), round(d['ms_per_step'],3), d['dtype'], c.get('fast_transactional'))"
}
for rep in 1 2; do
  run c3b_fused_$rep python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
  run c3b_generic_$rep SVOC_FUSED_TXN=0 python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
  run c3b_notxn_$rep python bench.py --config c3 --storage bf16 --transactional 0 --steps 20 --warmup 3
done
