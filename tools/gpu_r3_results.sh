#!/bin/bash
# Round-3 results session, part 2 (part 1 = the headline records of tools/gpu_results.sh): the wide /
# c1 records, kernel tables, then PMC of the fp32-storage window kernel at c3 and c2 (pmc.sh).
set -u
CFG=c3 EXTRA="--storage fp32" MEMSET="FETCH_SIZE" MEMSET2="WRITE_SIZE" bash tools/pmc.sh || exit 1
CFG=c2 EXTRA="--storage fp32" MEMSET="FETCH_SIZE" MEMSET2="WRITE_SIZE" bash tools/pmc.sh || exit 1
PART2=1 bash tools/gpu_results.sh || exit 1
echo all done
