set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wsad_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wsad_tests.log 2>&1; rc=$?; tail -15 gpurun_out/wsad_tests.log; [ $rc -ne 0 ] && exit $rc
for st in int32 int64; do
  timeout -k 10 300 python bench.py --config c2 --mode exact --storage $st --steps 10 --warmup 2 > gpurun_out/bench_exact_$st.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_exact_$st.log
done
SVOC_EXACT_I128=1 timeout -k 10 300 python bench.py --config c2 --mode exact --batch 2000 --steps 3 --warmup 1 > gpurun_out/bench_exact_i128.log 2>&1 || exit 1
tail -1 gpurun_out/bench_exact_i128.log
