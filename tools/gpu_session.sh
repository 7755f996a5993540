#!/bin/bash
# One GPU session: tests, benches, profile. Each GPU step has its own time limit; the script stops
# at the first crash / timeout (exit codes other than 0/1 from pytest, anything non-zero otherwise).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import torch; print(torch.__version__, torch.cuda.get_device_name(0))" || exit 3
stage() { echo "=== $1 ($(date +%T))"; }

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  stage pytest-gpu
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi

stage smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc

BENCHES="${BENCHES:-c2:10:2 c3:10:2}"
for spec in $BENCHES; do
  IFS=: read cfg steps warm <<< "$spec"
  stage "bench $cfg"
  timeout -k 10 400 python bench.py --config $cfg --steps $steps --warmup $warm > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; tail -3 gpurun_out/bench_$cfg.log; [ $rc -ne 0 ] && exit $rc
done

if [ -n "${PROFILE:-}" ]; then
  for cfg in $PROFILE; do
    stage "rocprof $cfg"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $R/gpurun_out/prof_$cfg -o run -- python3 $R/bench.py --config $cfg --steps 6 --warmup 1 --graph 0 \
        > $R/gpurun_out/prof_$cfg.log 2>&1)
    rc=$?; tail -3 gpurun_out/prof_$cfg.log; [ $rc -ne 0 ] && exit $rc
  done
fi
echo "=== done"
