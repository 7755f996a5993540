set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3xs -o run -- python3 $R/bench.py --config-file $R/configs/c3_exact_stream.yaml --steps 2 --warmup 1 --graph 0 > $R/gpurun_out/prof_c3xs.log 2>&1) || exit 1
head -14 gpurun_out/prof_c3xs/run_kernel_stats.csv | cut -d, -f1-7 | cut -c1-200
