#!/bin/bash
# Alternating A/B of bench lines under environment settings (same build):
#   AB_ENVS="SVOC_WINF_RAW=0|SVOC_WINF_RAW=1" AB_BENCH="--config c3 --storage fp32|--config c2 --storage fp32" \
#   REPS=2 bash tools/gpu_ab_env.sh
# Prints one line per (rep, env, bench): rounds/s and ms/step.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
IFS='|' read -ra ENVS <<< "${AB_ENVS:?}"
IFS='|' read -ra BS <<< "${AB_BENCH:?}"
for rep in $(seq 1 ${REPS:-2}); do
  for e in "${ENVS[@]}"; do
    for b in "${BS[@]}"; do
      env $e timeout -k 10 200 python bench.py $b --steps ${STEPS:-20} > gpurun_out/ab_env.log 2>&1 || { tail -5 gpurun_out/ab_env.log; exit 1; }
      python3 - "$rep" "$e" "$b" <<'EOF'
import json, sys
r = json.loads(open("gpurun_out/ab_env.log").read().strip().splitlines()[-1])
print(f"rep{sys.argv[1]} [{sys.argv[2]}] {sys.argv[3]}: {r['value']:.4g} rounds/s  {r['ms_per_step']:.3f} ms/step  ok={r['config'].get('ok_fraction')}")
EOF
    done
  done
done
