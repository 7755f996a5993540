# round 4: exact unconstrained + bf16 in-kernel rollback -- tests, then benches (A/B where noted)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_wsad_gpu.py tests/test_exact_stream.py tests/test_fast_transactional.py tests/test_win_gpu.py tests/test_win_gpu_extra.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_s2_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_s2_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag env... -- bench args
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r4_s2_$tag.log 2>&1 || { tail -5 gpurun_out/r4_s2_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_s2_$tag.log').read().strip().splitlines()[-1]); c=d['config']; print('$tag', round(d['value']), round(d['ms_per_step'],3), d['dtype'], c.get('ok_fraction'), c.get('fast_transactional'))"
}
for rep in 1 2; do
  run c3b_kroll_$rep python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
  run c3b_rkern_$rep SVOC_KERNEL_ROLLBACK=0 python bench.py --config c3 --storage bf16 --steps 20 --warmup 3
  run c3b_notxn_$rep python bench.py --config c3 --storage bf16 --transactional 0 --steps 20 --warmup 3
done
run c2u_col python bench.py --config-file configs/c2_exact_unconstrained.yaml --steps 10 --warmup 2
run c2u_i128 SVOC_EXACT_I128=1 python bench.py --config-file configs/c2_exact_unconstrained.yaml --steps 2 --warmup 1
run c2x_i64 python bench.py --config c2 --mode exact --storage int64 --steps 10 --warmup 2
run c2x_i32 python bench.py --config c2 --mode exact --steps 10 --warmup 2
run c3x python bench.py --config-file configs/c3_exact_rounds.yaml --steps 5 --warmup 1
bash tools/gpu_r4_c3b_trace.sh
