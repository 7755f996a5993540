#!/bin/bash
# MFMA / memory counters for the encoder kernels of the c4 config (kernel-trace + pmc only).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS" \
           "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "attn_short|add_layernorm|Cijk" \
     --output-format csv -d $R/gpurun_out/pmc_c4_$i -o run -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --graph 0 \
     > $R/gpurun_out/pmc_c4_$i.log 2>&1) || { echo "pmc set $i failed"; tail -5 gpurun_out/pmc_c4_$i.log; }
done
echo done
