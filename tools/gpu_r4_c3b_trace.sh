# round 4: kernel trace of the c3 bf16 step, transactional (generic path) vs not
set -u
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
for t in 1 0; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d $R/gpurun_out/trace_c3b_t$t -o run -- python3 $R/bench.py --config c3 --storage bf16 --transactional $t --steps 8 --warmup 2 --graph 0 \
     > $R/gpurun_out/trace_c3b_t$t.log 2>&1) || { echo "trace failed"; tail -5 gpurun_out/trace_c3b_t$t.log; exit 1; }
  python3 tools/trace_step.py gpurun_out/trace_c3b_t$t consensus_fast > gpurun_out/trace_c3b_t$t.md
  echo "== transactional $t"; cat gpurun_out/trace_c3b_t$t.md
done
