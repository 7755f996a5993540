#!/bin/bash
# A/B of the N <= 64 window kernel's waves per workgroup on c2, alternating.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for w in 4 2 8; do
    SVOC_WIN_WAVES=$w timeout -k 10 120 python bench.py --config c2 --steps 20 --warmup 3 > gpurun_out/wc2_${w}_$rep.log 2>&1 || exit 1
    python - "$w" "$rep" <<'PY'
import json, sys
w, rep = sys.argv[1:]
line = [l for l in open(f"gpurun_out/wc2_{w}_{rep}.log").read().splitlines() if l.startswith("{")][-1]
d = json.loads(line)
print(json.dumps(dict(config="c2", waves=int(w), rep=int(rep), rounds_per_s=d["value"], ms_per_step=d["ms_per_step"])))
PY
  done
done | tee gpurun_out/waves_c2.jsonl
