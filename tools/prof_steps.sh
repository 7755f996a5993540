#!/bin/bash
# Kernel trace of steady-state bench steps (graph replay off so every kernel is a separate dispatch).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
for spec in ${CFGS:-c3:12}; do
  IFS=: read cfg steps <<< "$spec"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
     -d $R/gpurun_out/trace_$cfg -o run -- python3 $R/bench.py --config $cfg --steps $steps --warmup 2 --graph 0 \
     > $R/gpurun_out/trace_$cfg.log 2>&1) || { echo "trace $cfg failed"; tail -5 gpurun_out/trace_$cfg.log; exit 1; }
  python3 tools/trace_step.py gpurun_out/trace_$cfg ${ANCHOR:-consensus_fast} > gpurun_out/trace_${cfg}.md
  cat gpurun_out/trace_${cfg}.md
done
