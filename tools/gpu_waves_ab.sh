#!/bin/bash
# A/B of the window kernel's waves per workgroup on c3 (pipeline ranges x waves), alternating.
# usage: tools/gpu_waves_ab.sh "4 8 16" "1 2 4" reps
set -u
mkdir -p gpurun_out
WS=${1:-"4 8"}; PLS=${2:-"2 1"}; REPS=${3:-2}
for rep in $(seq $REPS); do
  for w in $WS; do
    for pl in $PLS; do
      SVOC_WIN_WAVES=$w timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --pipeline $pl > gpurun_out/wab_${w}_${pl}_$rep.log 2>&1 || exit 1
      python - "$w" "$pl" "$rep" <<'PY'
import json, sys
w, pl, rep = sys.argv[1:]
line = [l for l in open(f"gpurun_out/wab_{w}_{pl}_{rep}.log").read().splitlines() if l.startswith("{")][-1]
d = json.loads(line)
print(json.dumps(dict(waves=int(w), pipeline=int(pl), rep=int(rep), rounds_per_s=d["value"], ms_per_step=d["ms_per_step"])))
PY
    done
  done
done | tee gpurun_out/waves_ab.jsonl
