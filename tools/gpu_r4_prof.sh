# round 4: where the c3 fp32 step goes -- kernel traces of rounds-only and streaming, both window configs
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
p() {  # tag, cfg, bench args
  local tag=$1 cfg=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp && SVOC_WINF_CFG=$cfg timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/gpurun_out/prof_$tag -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/prof_$tag.log 2>&1) || { tail -5 gpurun_out/prof_$tag.log; exit 1; }
  tail -1 gpurun_out/prof_$tag.log | cut -c1-200
  python3 tools/prof_summary.py gpurun_out/prof_$tag 2>/dev/null | head -12 || true
}
p r4x1 4x1 --config-file $R/configs/c3_rounds.yaml --steps 6 --warmup 1 --graph 0
p r2x2 2x2 --config-file $R/configs/c3_rounds.yaml --steps 6 --warmup 1 --graph 0
p s4x1t1 4x1 --storage fp32 --steps 6 --warmup 1 --transactional 1
p s4x1t0 4x1 --storage fp32 --steps 6 --warmup 1 --transactional 0
