# round 4: double-buffered LDS-DMA window kernel (SVOC_WINF_CFG default 2x2 vs 4x1) -- tests, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_f32_gpu.py tests/test_fast_transactional.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_dbuf_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_dbuf_tests.log; [ $rc -eq 0 ] || exit $rc
SVOC_WINF_CFG=4x1 timeout -k 10 600 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread -k "window or pruned" > gpurun_out/r4_dbuf_tests_4x1.log 2>&1; rc=$?; tail -2 gpurun_out/r4_dbuf_tests_4x1.log; [ $rc -eq 0 ] || exit $rc
b() {  # tag, env cfg, bench args
  local tag=$1 cfg=$2; shift 2
  SVOC_WINF_CFG=$cfg timeout -k 10 300 python bench.py "$@" > gpurun_out/r4_ab_$tag.log 2>&1 || { tail -5 gpurun_out/r4_ab_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_ab_$tag.log').read().splitlines()[-1]); c=d['config']; print('$tag', round(d['value']), round(d['ms_per_step'],3), c.get('fast_transactional'), c.get('pruned_net_fallback_rate'))"
}
for r in 1 2; do
  b c3_2x2_t0_$r 2x2 --storage fp32 --transactional 0
  b c3_4x1_t0_$r 4x1 --storage fp32 --transactional 0
  b c3_2x2_t1_$r 2x2 --storage fp32 --transactional 1
  b c3_4x1_t1_$r 4x1 --storage fp32 --transactional 1
done
b c2f_2x2 2x2 --config c2 --storage fp32
b c2f_4x1 4x1 --config c2 --storage fp32
