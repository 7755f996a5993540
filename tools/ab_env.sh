#!/bin/bash
# A/B of an environment switch on one build, alternating on one box:
#   AB_ENV=SVOC_LEAN_COMMIT AB_VALUES="0 1" AB_CONFIGS="--config c3" AB_REPS=4 bash tools/ab_env.sh
set -u
mkdir -p gpurun_out
CONFIGS="${AB_CONFIGS:---config c3}"
REPS="${AB_REPS:-3}"
IFS='|' read -ra CFGS <<< "$CONFIGS"
for rep in $(seq 1 $REPS); do
  for v in ${AB_VALUES:-0 1}; do
    for cfg in "${CFGS[@]}"; do
      tag=$(echo $cfg | tr -cd 'a-z0-9')
      env "$AB_ENV=$v" timeout -k 10 200 python bench.py $cfg --steps 30 --warmup 3 > gpurun_out/abe_${v}_${tag}_$rep.log 2>&1 || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/abe_${v}_${tag}_$rep.log').read().strip().splitlines()[-1]); print('$AB_ENV=$v $tag rep$rep', round(d['value']), round(d['ms_per_step'],4))"
    done
  done
done
