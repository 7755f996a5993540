#!/bin/bash
# Two ranks of bench.py on ONE MI355X over gloo, each started directly under rocprofv3 --kernel-trace (RANK /
# WORLD_SIZE exported here, no launcher hop): the per-process kernel timelines of the multi-rank bench path
# (VERDICT r4 item 5b).  Then tools/two_rank_timeline.py merges them.
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 WORLD_SIZE=2 LOCAL_RANK=0 HSA_ENABLE_IPC_MODE_LEGACY=0
STOR=${STOR:-fp32}
for r in 0 1; do
  (cd /tmp && export TMPDIR=/tmp RANK=$r && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d $R/gpurun_out/tr_${STOR}_r$r -o run -- python3 $R/bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo \
     --storage $STOR ${EXTRA:-} > $R/gpurun_out/tr_${STOR}_r$r.log 2>&1) &
done
wait
grep -h '^{' gpurun_out/tr_${STOR}_r0.log | cut -c1-300
python3 tools/two_rank_timeline.py gpurun_out/tr_${STOR}_r0 gpurun_out/tr_${STOR}_r1 > gpurun_out/tr_${STOR}_timeline.txt
cat gpurun_out/tr_${STOR}_timeline.txt
