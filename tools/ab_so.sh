#!/bin/bash
# A/B of two builds of svoc/_C.so (old = HEAD, new = working tree), alternating, one box.
# usage: build HEAD and the working tree into ab/_C_old.so and ab/_C_new.so first (csrc/build.py + cp)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_win_gpu.py tests/test_win_gpu_extra.py -x -q --timeout 120 --timeout-method thread > gpurun_out/win_tests.log 2>&1 || exit 1; tail -1 gpurun_out/win_tests.log
for rep in 1 2 3; do
  for v in old new; do
    cp ab/_C_$v.so svoc/_C.so
    for cfg in "--config c2" "--config-file configs/ab_c128.yaml"; do
      tag=$(echo $cfg | tr -cd 'a-z0-9')
      timeout -k 10 200 python bench.py $cfg --steps 30 --warmup 3 > gpurun_out/ab_${v}_${tag}_$rep.log 2>&1 || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/ab_${v}_${tag}_$rep.log').read().strip().splitlines()[-1]); print('$v $tag rep$rep', round(d['value']), round(d['ms_per_step'],4))"
    done
  done
done
cp ab/_C_new.so svoc/_C.so
