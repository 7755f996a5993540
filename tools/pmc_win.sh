#!/bin/bash
# PMC passes of the window kernels (c3 fp32 + c2 bf16): the two SQ sets of tools/pmc.sh plus the L2 hit / miss and
# HBM fetch sets, then one summary per config over every pass directory pmc.sh wrote.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for cfg in c3 c2; do
  CFG=$cfg MEMSET="TCC_HIT_sum TCC_MISS_sum" MEMSET2="FETCH_SIZE" bash tools/pmc.sh || exit 1
  python tools/pmc_summary.py gpurun_out/pmc_${cfg}_[0-9]* > gpurun_out/pmc_${cfg}_win.txt || exit 1
done
