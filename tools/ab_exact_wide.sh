# A/B of two builds of svoc/_C.so for the i128 exact kernel (build them into ab/ first, as for ab_so.sh):
#   bash tools/ab_exact_wide.sh   -> old/new rounds/s for configs/wide4096_exact.yaml and c5 exact, then the exact GPU tests
set -u
for rep in 1 2; do for v in old new; do
  cp ab/_C_$v.so svoc/_C.so
  timeout -k 10 200 python bench.py --config-file configs/wide4096_exact.yaml --steps 1 --warmup 1 > gpurun_out/abx_w_$v$rep.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --config-file configs/c5_exact_rounds.yaml --steps 20 --warmup 2 > gpurun_out/abx_c5_$v$rep.log 2>&1 || exit 1
  python -c "
import json
for t in ('w','c5'):
    d=json.loads(open('gpurun_out/abx_'+t+'_$v$rep.log').read().strip().splitlines()[-1]); print('$v', t, 'rep$rep', round(d['value'],1), round(d['ms_per_step'],3))"
done; done
cp ab/_C_new.so svoc/_C.so
timeout -k 10 400 python -u -m pytest tests/test_wide_gpu.py tests/test_ops_gpu.py tests/test_legacy.py tests/test_governance_gpu.py tests/test_wsad_gpu.py tests/test_revert_gpu.py tests/test_exact_stream.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/abx_tests.log 2>&1; tail -1 gpurun_out/abx_tests.log
