cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config-file $R/configs/wide512_exact.yaml --steps 3 --warmup 1 > gpurun_out/b_w512x.log 2>&1 || { tail -5 gpurun_out/b_w512x.log; exit 1; }
grep '^{' gpurun_out/b_w512x.log | cut -c1-220
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_w4096x -o run -- python3 $R/bench.py --config-file $R/configs/wide4096_exact.yaml --steps 3 --warmup 1 --graph 0 > $R/gpurun_out/prof_w4096x.log 2>&1) || exit 1
head -8 gpurun_out/prof_w4096x/run_kernel_stats.csv | cut -c1-200
