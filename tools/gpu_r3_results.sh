#!/bin/bash
# Round-3 results session on the committed tree: full GPU test suite, smoke, then every headline bench
# record + kernel tables (tools/gpu_results.sh).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_gputest.log 2>&1 || { tail -30 gpurun_out/r3_gputest.log; exit 1; }
tail -1 gpurun_out/r3_gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -5 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
bash tools/gpu_results.sh || exit 1
echo all done
