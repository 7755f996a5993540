# Exact transactional waves in the update / restore kernels: the stream tests, then the exact stream benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_exact_stream.py tests/test_fast_transactional.py tests/test_revert_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_xtx.log 2>&1; rc=$?; tail -3 gpurun_out/pt_xtx.log; [ $rc -ne 0 ] && exit $rc
for spec in "c3xs:--config-file configs/c3_exact_stream.yaml --steps 2 --warmup 1" "c3xsi:--config-file configs/c3_exact_stream_indep.yaml --steps 2 --warmup 1" "c5xs:--config-file configs/c5_exact_stream.yaml --steps 20 --warmup 2"; do
  k=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python bench.py $a > gpurun_out/b_$k.log 2>&1 || { tail -5 gpurun_out/b_$k.log; exit 1; }
  echo "$k $(grep '^{' gpurun_out/b_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'], d['config'].get('ok_fraction'))")"
done
