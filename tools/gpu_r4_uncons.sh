# round 4: unconstrained rounds in the exact column kernel -- tests, then the c2-shape unconstrained bench
# (column kernel vs SVOC_EXACT_I128=1) and the constrained exact configs (no regression)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wsad_gpu.py tests/test_exact_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_uncons_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_uncons_tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag env... -- bench args
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r4_uncons_$tag.log 2>&1 || { tail -5 gpurun_out/r4_uncons_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_uncons_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']), round(d['ms_per_step'],3), d['dtype'], d['config'].get('ok_fraction'))"
}
run c2u_col python bench.py --config-file configs/c2_exact_unconstrained.yaml --steps 10 --warmup 2
run c2u_col_i32cmp python bench.py --config c2 --mode exact --storage int64 --steps 10 --warmup 2
run c2u_i128 SVOC_EXACT_I128=1 python bench.py --config-file configs/c2_exact_unconstrained.yaml --steps 2 --warmup 1
run c2x_i32 python bench.py --config c2 --mode exact --steps 10 --warmup 2
run c3x python bench.py --config-file configs/c3_exact_rounds.yaml --steps 5 --warmup 1
