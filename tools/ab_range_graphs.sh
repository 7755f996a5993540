#!/bin/bash
# c3 fp32 transactional: one graph for both pipelined ranges (default) vs one linear graph per range (--range-graphs 1).
# (the --range-graphs flag was removed after this A/B: profiles/r5_c3_range_graphs_ab.txt, docs/PERF.md)
set -u
for rep in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 --range-graphs $v > gpurun_out/abrg_$v.log 2>&1 || { tail -5 gpurun_out/abrg_$v.log; exit 1; }
    python - $v $rep <<'P'
import json,sys
l=[x for x in open(f"gpurun_out/abrg_{sys.argv[1]}.log") if x.startswith("{")][-1]; d=json.loads(l)
print("range_graphs", sys.argv[1], "rep", sys.argv[2], round(d["value"]), round(d["ms_per_step"],4), "ok", d["config"].get("ok_fraction"), "rg", d["config"].get("range_graphs", d.get("range_graphs")))
P
  done
done
