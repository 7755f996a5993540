#!/bin/bash
# Kernel stats + PMC of the consensus kernels for bench configs.
#   SPECS="c3:--storage fp32 --pipeline 1;c2:--storage fp32" bash tools/gpu_prof.sh
# Per spec: one rocprofv3 --kernel-trace --stats run (graph replay off: every kernel a dispatch), then
# PMC passes (kernel-trace + pmc only), each in its own run: SQ issue/wait counters, FETCH_SIZE,
# WRITE_SIZE.  Outputs under gpurun_out/prof_<tag>/ and a summary in gpurun_out/prof_<tag>.md.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
KRE=${KRE:-consensus_fast|upd_|apply}
IFS=';' read -ra SP <<< "${SPECS:-c3:--storage fp32 --pipeline 1}"
n=0
for spec in "${SP[@]}"; do
  n=$((n+1))
  cfg=${spec%%:*}; extra=${spec#*:}
  tag=${cfg}_$n
  out=$R/gpurun_out/prof_$tag; mkdir -p $out
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $out/stats -o run -- python3 $R/bench.py --config $cfg --steps ${STEPS:-6} --warmup 2 --graph 0 $extra \
     > $out/stats.log 2>&1) || { echo "stats $tag failed"; tail -5 $out/stats.log; exit 1; }
  python3 tools/prof_summary.py $out/stats $R/gpurun_out/prof_$tag.md > /dev/null
  if [ "${PMC:-1}" = "1" ]; then
    i=0
    for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM" \
               "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$KRE" \
         --output-format csv -d $out/pmc_$i -o run -- python3 $R/bench.py --config $cfg --steps 2 --warmup 1 --graph 0 $extra \
         > $out/pmc_$i.log 2>&1) || { echo "pmc $tag set $i failed"; tail -5 $out/pmc_$i.log; exit 1; }
    done
    python3 tools/pmc_summary.py $out/pmc_* >> $R/gpurun_out/prof_$tag.md 2>&1 || true
  fi
  echo "== $tag ($spec)"; cat $R/gpurun_out/prof_$tag.md
done
