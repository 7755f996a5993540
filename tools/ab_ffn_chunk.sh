cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for rep in 1 2; do
for ch in 0 16384 32768 65536; do
  SVOC_FFN_CHUNK=$ch timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/ffn_$ch.log 2>&1 || exit 1
  echo "chunk $ch: $(grep -o '"value": [0-9.]*' gpurun_out/ffn_$ch.log | head -1) $(grep -o '"alt_precision": {"encoder_dtype": "fp32", "value": [0-9.]*' gpurun_out/ffn_$ch.log)"
done; done
