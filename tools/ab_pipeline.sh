#!/bin/bash
# c3 fp32 transactional: instance ranges per pipelined step (bench.py --pipeline), alternating on one box.
set -u
for rep in 1 2; do
  for k in 2 4 3; do
    timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 --pipeline $k > gpurun_out/abpl_$k.log 2>&1 || { tail -5 gpurun_out/abpl_$k.log; exit 1; }
    python - $k $rep <<'P'
import json,sys
l=[x for x in open(f"gpurun_out/abpl_{sys.argv[1]}.log") if x.startswith("{")][-1]; d=json.loads(l)
alt=d["config"].get("alt_storage")
print("pipeline", sys.argv[1], "rep", sys.argv[2], round(d["value"]), round(d["ms_per_step"],4), "alt", round(alt["value"]) if isinstance(alt, dict) else alt)
P
  done
done
