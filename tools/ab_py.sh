#!/bin/bash
set -u
for rep in 1 2 3; do
  for v in old new; do
    b=bench.py; [ $v = old ] && b=ab/bench.py
    timeout -k 10 200 python $b --config c2 --steps 20 --warmup 3 > gpurun_out/abp_$v.log 2>&1 || { tail -5 gpurun_out/abp_$v.log; exit 1; }
    python - $v $rep <<'P'
import json,sys
l=[x for x in open(f"gpurun_out/abp_{sys.argv[1]}.log") if x.startswith("{")][-1]; d=json.loads(l)
print(sys.argv[1], "rep", sys.argv[2], round(d["value"]), round(d["ms_per_step"],4), "alt", round(d["config"]["alt_storage"]["value"]) if isinstance(d["config"].get("alt_storage"),dict) else d["config"].get("alt_storage"), d.get("graph_steps", d["config"].get("graph_steps")))
P
  done
done
