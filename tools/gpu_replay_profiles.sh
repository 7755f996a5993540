#!/bin/bash
# Timed-region kernel tables: rocprofv3 kernel traces of bench.py --markers for c3 (fp32
# headline, bf16 alt_storage, exact stream), c2 (bf16, fp32 alt) and c4 (bf16, fp32 alt_precision, cls head),
# rendered by tools/replay_kernels.py into gpurun_out/replay_*.md.  Each GPU step has its own time limit; the
# script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {   # config, steps
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv \
      -d "$R/gpurun_out/rk_$1" -o run -- python3 "$R/bench.py" --config "$1" --steps "$2" --warmup 3 --markers \
      > "$R/gpurun_out/rk_$1.log" 2>&1)
  rc=$?; tail -1 "gpurun_out/rk_$1.log" | cut -c1-300; return $rc
}
run c3 20 || exit $?
python3 tools/replay_kernels.py gpurun_out/rk_c3 "c3 fp32 transactional (headline), timed replay only" 1 20 > gpurun_out/replay_c3_fp32.md
python3 tools/replay_kernels.py gpurun_out/rk_c3 "c3 bf16 storage (alt_storage), timed replay only" 2 20 > gpurun_out/replay_c3_bf16.md
python3 tools/replay_kernels.py gpurun_out/rk_c3 "c3 exact transactional stream (exact_stream), timed steps only" 3 2 > gpurun_out/replay_c3_exact_stream.md
run c2 20 || exit $?
python3 tools/replay_kernels.py gpurun_out/rk_c2 "c2 bf16, timed replay only" 1 20 > gpurun_out/replay_c2_bf16.md
python3 tools/replay_kernels.py gpurun_out/rk_c2 "c2 fp32 storage (alt_storage), timed replay only" 2 20 > gpurun_out/replay_c2_fp32.md
run c4 10 || exit $?
python3 tools/replay_kernels.py gpurun_out/rk_c4 "c4 bf16 (mean pooling), timed steps only" 1 10 > gpurun_out/replay_c4_bf16.md
python3 tools/replay_kernels.py gpurun_out/rk_c4 "c4 fp32 (alt_precision), timed steps only" 2 10 > gpurun_out/replay_c4_fp32.md
python3 tools/replay_kernels.py gpurun_out/rk_c4 "c4 bf16, <s> classifier head (cls_pool), timed steps only" 3 10 > gpurun_out/replay_c4_cls.md
rm -rf gpurun_out/rk_c2 gpurun_out/rk_c3 gpurun_out/rk_c4
echo "=== done"
