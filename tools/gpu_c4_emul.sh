# fp32 GEMMs emulated on the bf16 matrix cores: encoder GPU tests, then c4 with the emulated and native fp32 GEMMs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_encoder_ops_gpu.py tests/test_sentiment.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_enc.log 2>&1; rc=$?; tail -15 gpurun_out/pt_enc.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/b_c4_emul.log 2>&1 || { tail -5 gpurun_out/b_c4_emul.log; exit 1; }
grep '^{' gpurun_out/b_c4_emul.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', round(d['value']), d['config']['alt_precision'])"
SVOC_FP32_GEMM=native timeout -k 10 400 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/b_c4_native.log 2>&1 || { tail -5 gpurun_out/b_c4_native.log; exit 1; }
grep '^{' gpurun_out/b_c4_native.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 native', round(d['value']), d['config']['alt_precision'])"
