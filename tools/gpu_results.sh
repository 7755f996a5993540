#!/bin/bash
# Every headline bench record on one MI355X -> profiles/results.jsonl (one source of truth for the
# README / BASELINE tables: python tools/results_table.py), plus the c2 / c3 rocprofv3 kernel tables.
set -u
R=$(pwd)
mkdir -p gpurun_out
OUT=gpurun_out/results.jsonl
: > $OUT
run() {  # key, timeout, bench args...
  local key=$1 t=$2; shift 2
  echo "=== $key ($(date +%T))"
  timeout -k 10 $t python bench.py "$@" > gpurun_out/res_$key.log 2>&1 || { tail -5 gpurun_out/res_$key.log; return 1; }
  python - "$key" <<'PY' >> $OUT
import json, sys
line = [l for l in open(f"gpurun_out/res_{sys.argv[1]}.log").read().splitlines() if l.startswith("{")][-1]
d = json.loads(line); d["key"] = sys.argv[1]; print(json.dumps(d))
PY
  tail -1 $OUT | cut -c1-160
}
if [ -z "${PART2:-}" ]; then
run c3 400 --config c3 --steps 20 --warmup 3 &&
run c3_notxn 300 --config c3 --storage fp32 --transactional 0 --steps 20 --warmup 3 &&
run c3_bf16 300 --config c3 --storage bf16 --steps 20 --warmup 3 &&
run c2 300 --config c2 --steps 20 --warmup 3 &&
run c2_fp32 300 --config c2 --storage fp32 --steps 20 --warmup 3 &&
run c5 300 --config c5 --steps 50 --warmup 3 &&
run c4 300 --config c4 --steps 10 --warmup 2 &&
run c2_exact 300 --config c2 --mode exact --steps 10 --warmup 2 &&
run c2_exact_int64 300 --config c2 --mode exact --storage int64 --steps 10 --warmup 2 &&
run c5_exact 300 --config-file configs/c5_exact_rounds.yaml --steps 20 --warmup 2 &&
run c3_exact 300 --config-file configs/c3_exact_rounds.yaml --steps 10 --warmup 2 &&
run c2_exact_uncons 300 --config-file configs/c2_exact_unconstrained.yaml --steps 10 --warmup 2 &&
run c2_exact_uncons_prices 300 --config-file configs/c2_exact_unconstrained_prices.yaml --steps 10 --warmup 2 &&
run c2_exact_uncons_wide 300 --config-file configs/c2_exact_unconstrained_wide.yaml --steps 10 --warmup 2 &&
run c5_exact_stream 300 --config-file configs/c5_exact_stream.yaml --steps 20 --warmup 2 &&
true || exit 1
fi
run wide512 300 --config-file configs/wide512.yaml --steps 10 --warmup 2 &&
run wide512_fp32 300 --config-file configs/wide512.yaml --storage fp32 --steps 10 --warmup 2 &&
run wide2048 300 --config-file configs/wide2048.yaml --steps 5 --warmup 1 &&
run wide2048_fp32 300 --config-file configs/wide2048.yaml --storage fp32 --steps 5 --warmup 1 &&
run wide512_exact 300 --config-file configs/wide512_exact.yaml --steps 3 --warmup 1 &&
run wide4096_exact 300 --config-file configs/wide4096_exact.yaml --steps 3 --warmup 1 &&
run wide4096_exact_dshard 300 --config-file configs/wide4096_exact.yaml --dshard --steps 3 --warmup 1 &&
run c1 300 --config c1 --steps 50 --warmup 3 || exit 1
# (kernel tables of the timed replay only: tools/gpu_replay_profiles.sh)
# last: 64 exact transactions per instance per step at the YAML batch (1024 instances)
run c3_exact_stream 150 --config-file configs/c3_exact_stream.yaml --steps 2 --warmup 1 &&
run c3_exact_stream_indep 150 --config-file configs/c3_exact_stream_indep.yaml --steps 2 --warmup 1 || exit 1
echo "=== done"
