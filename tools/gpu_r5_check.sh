# Round-5 kernel check: exact / transactional / wide GPU tests, then the exact and c3 headline benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; R=$(pwd); mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_wsad_gpu.py tests/test_ops_gpu.py tests/test_revert_gpu.py tests/test_exact_stream.py tests/test_fast_transactional.py tests/test_wide_gpu.py tests/test_f32_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_r5.log 2>&1; rc=$?; tail -3 gpurun_out/pt_r5.log; [ $rc -ne 0 ] && exit $rc
for spec in "c3:" "c3x:--config-file configs/c3_exact_rounds.yaml --steps 10 --warmup 2" "c2x:--config c2 --mode exact --steps 10 --warmup 2" "c2u:--config-file configs/c2_exact_unconstrained.yaml --steps 10 --warmup 2" "c2up:--config-file configs/c2_exact_unconstrained_prices.yaml --steps 10 --warmup 2" "c2x64:--config c2 --mode exact --storage int64 --steps 10 --warmup 2" "w512x:--config-file configs/wide512_exact.yaml --steps 3 --warmup 1" "w4096x:--config-file configs/wide4096_exact.yaml --steps 3 --warmup 1"; do
  k=${spec%%:*}; a=${spec#*:}
  timeout -k 10 400 python bench.py $a > gpurun_out/b_$k.log 2>&1 || { tail -5 gpurun_out/b_$k.log; exit 1; }
  echo "$k $(grep '^{' gpurun_out/b_$k.log | tail -1 | cut -c1-160)"
done
