# round 4: update kernel split (save path in its own instantiation) -- tests, c3 bf16 / fp32 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fast_transactional.py tests/test_ops_gpu.py tests/test_revert_gpu.py tests/test_pipeline_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_s3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_s3_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag env... -- bench args
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r4_s3_$tag.log 2>&1 || { tail -5 gpurun_out/r4_s3_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_s3_$tag.log').read().strip().splitlines()[-1]); c=d['config']; print('$tag', round(d['value']), round(d['ms_per_step'],3), d['dtype'], c.get('fast_transactional'), c.get('alt_storage'))"
}
for rep in 1 2; do
  run c3b_kroll_$rep python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
  run c3b_rkern_$rep SVOC_KERNEL_ROLLBACK=0 python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
  run c3b_notxn_$rep python bench.py --config c3 --storage bf16 --transactional 0 --steps 20 --warmup 3
  run c3f_$rep python bench.py --config c3 --steps 20 --warmup 3
done
bash tools/gpu_r4_c3b_trace.sh
