#!/bin/bash
# Quick check after a kernel change: GPU tests, then the headline benches (one line each).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_gputest.log 2>&1 || { tail -30 gpurun_out/q_gputest.log; exit 1; }
tail -1 gpurun_out/q_gputest.log
b() { timeout -k 10 200 python bench.py "$@" > gpurun_out/q_b.log 2>&1 || { tail -5 gpurun_out/q_b.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/q_b.log') if l.startswith('{')][-1]); a=d['config'].get('alt_storage') or {}; print(sys.argv[1:], round(d['value']), d['ms_per_step'], 'alt', a.get('value'))" "$@"; }
b --config c3 --steps 20 --warmup 3
b --config c3 --steps 20 --warmup 3 --pipeline 1
b --config c3 --steps 20 --warmup 3 --pipeline 4
b --config c2 --steps 20 --warmup 3
echo done
