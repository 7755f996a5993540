#!/bin/bash
# PMC counters for the consensus kernels (kernel-trace + pmc only; no sys/runtime traces).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
CFG=${CFG:-c2}
KRE=${KRE:-consensus_fast}                 # kernel name regex
ARGS=${ARGS:---config $CFG}                # bench.py config arguments (e.g. --config-file configs/X.yaml)
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
      "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_VMEM")
[ -n "${MEMSET:-}" ] && SETS+=("$MEMSET")
[ -n "${MEMSET2:-}" ] && SETS+=("$MEMSET2")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex $KRE \
     --output-format csv -d $R/gpurun_out/pmc_${CFG}_$i -o run -- python3 $R/bench.py $ARGS --steps 3 --warmup 1 --graph 0 ${EXTRA:-} \
     > $R/gpurun_out/pmc_${CFG}_$i.log 2>&1) || { echo "pmc set $i failed"; tail -5 gpurun_out/pmc_${CFG}_$i.log; exit 1; }
done
echo done
