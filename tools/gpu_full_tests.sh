# Every GPU test + smoke (the driver's round-end tiers), then a c3 bf16 kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_all.log 2>&1; rc=$?; tail -4 gpurun_out/pt_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/prof_c3bf16 -o run -- python3 $R/bench.py --config c3 --storage bf16 --steps 6 --warmup 1 --graph 0 \
    > $R/gpurun_out/prof_c3bf16.log 2>&1) || exit 1
head -12 gpurun_out/prof_c3bf16/run_kernel_stats.csv | cut -c1-160
