#!/bin/bash
# PMC passes of the exact column kernel (consensus_wsad.hip) on the c3 and c2 exact configs, then the summary.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
CFG=c3x KRE=consensus_wsad ARGS="--config-file $(pwd)/configs/c3_exact_rounds.yaml" bash tools/pmc.sh || exit 1
CFG=c2x KRE=consensus_wsad ARGS="--config c2 --mode exact" bash tools/pmc.sh || exit 1
python tools/pmc_summary.py gpurun_out/pmc_c3x_1 gpurun_out/pmc_c3x_2 > gpurun_out/pmc_c3x.txt
python tools/pmc_summary.py gpurun_out/pmc_c2x_1 gpurun_out/pmc_c2x_2 > gpurun_out/pmc_c2x.txt
cat gpurun_out/pmc_c3x.txt gpurun_out/pmc_c2x.txt
