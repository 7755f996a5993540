#!/bin/bash
# A/B of builds of svoc/_C.so (ab/_C_<variant>.so; default variants: old new), alternating on one box.
# usage: build them into ab/ first (csrc/build.py + cp), then
#   AB_VARIANTS="old v1 new" AB_CONFIGS="--config c3|--config c2" AB_REPS=3 bash tools/ab_so.sh
set -u
mkdir -p gpurun_out
CONFIGS="${AB_CONFIGS:---config c2|--config-file configs/ab_c128.yaml}"
REPS="${AB_REPS:-3}"
VARS="${AB_VARIANTS:-old new}"
TESTV="${AB_TEST_VARIANT:-${VARS##* }}"   # the build the tests run on (default: the last variant)
if [ "${AB_TESTS:-1}" = "1" ]; then
  cp ab/_C_$TESTV.so svoc/_C.so
  timeout -k 10 300 python -u -m pytest ${AB_TEST_FILES:-tests/test_win_gpu.py tests/test_win_gpu_extra.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/win_tests.log 2>&1 || { tail -5 gpurun_out/win_tests.log; exit 1; }; tail -1 gpurun_out/win_tests.log
fi
IFS='|' read -ra CFGS <<< "$CONFIGS"
for rep in $(seq 1 $REPS); do
  for v in $VARS; do
    cp ab/_C_$v.so svoc/_C.so
    for cfg in "${CFGS[@]}"; do
      tag=$(echo $cfg | tr -cd 'a-z0-9')
      timeout -k 10 200 python bench.py $cfg --steps 30 --warmup 3 > gpurun_out/ab_${v}_${tag}_$rep.log 2>&1 || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/ab_${v}_${tag}_$rep.log').read().strip().splitlines()[-1]); print('$v $tag rep$rep', round(d['value']), round(d['ms_per_step'],4))"
    done
  done
done
cp ab/_C_$TESTV.so svoc/_C.so
