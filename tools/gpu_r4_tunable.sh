# round 4: c4 GEMMs with PyTorch TunableOp (hipBLASLt / rocBLAS solutions benchmarked per shape) vs the
# library heuristics; the tuned table is written to gpurun_out/tunableop_c4*.csv
set -o pipefail
mkdir -p gpurun_out
run() {  # tag env... -- bench args
  local tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/r4_tun_$tag.log 2>&1 || { tail -5 gpurun_out/r4_tun_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_tun_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), round(d['ms_per_step'],2), d['config'].get('alt_precision'))"
}
run base1 python bench.py --config c4 --steps 10 --warmup 3
run tune PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_c4.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=100 python bench.py --config c4 --steps 10 --warmup 4
ls gpurun_out/tunableop_c4* && head -30 gpurun_out/tunableop_c4*.csv
run tuned PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_c4.csv python bench.py --config c4 --steps 10 --warmup 3
run base2 python bench.py --config c4 --steps 10 --warmup 3
