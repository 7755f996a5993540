set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32_tests.log 2>&1
rc=$?; tail -30 gpurun_out/f32_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python bench.py --config c2 --storage fp32 --steps 20 --warmup 3 > gpurun_out/f32_c2.log 2>&1 || { tail gpurun_out/f32_c2.log; exit 1; }
tail -1 gpurun_out/f32_c2.log
timeout -k 10 200 python bench.py --config c3 --storage fp32 --steps 20 --warmup 3 > gpurun_out/f32_c3.log 2>&1 || { tail gpurun_out/f32_c3.log; exit 1; }
tail -1 gpurun_out/f32_c3.log
R=$(pwd)
for cfg in c2 c3; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/gpurun_out/prof_f32_$cfg -o run -- python3 $R/bench.py --config $cfg --storage fp32 --steps 6 --warmup 1 --graph 0 \
      > $R/gpurun_out/prof_f32_$cfg.log 2>&1) || exit 1
done
echo "=== done"
