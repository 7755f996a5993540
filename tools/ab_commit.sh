#!/bin/bash
# A/B of the fused fp32 transactional step's commit: the round kernel's own (default) vs the separate commit kernel.
set -u
for rep in 1 2 3; do
  for v in kernel round; do
    SVOC_FUSED_COMMIT=$v timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 > gpurun_out/abc_$v.log 2>&1 || { tail -5 gpurun_out/abc_$v.log; exit 1; }
    python - $v $rep <<'P'
import json,sys
l=[x for x in open(f"gpurun_out/abc_{sys.argv[1]}.log") if x.startswith("{")][-1]; d=json.loads(l)
print(sys.argv[1], "rep", sys.argv[2], round(d["value"]), round(d["ms_per_step"],4), "ok", d["config"].get("ok_fraction"))
P
  done
done
