# round 4: exact column kernel with the reliable-outlier int64 path: tests, then the exact c3 streams
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wsad_gpu.py tests/test_exact_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_exact_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_exact_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in c3_exact_stream c3_exact_stream_indep; do
  timeout -k 10 400 python -u bench.py --config-file configs/$cfg.yaml --steps 2 --warmup 1 > gpurun_out/r4_$cfg.log 2>&1 || { tail -5 gpurun_out/r4_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_$cfg.log').read().splitlines()[-1]); print('$cfg', round(d['value']), round(d['ms_per_step'],1), d['config'].get('ok_fraction'))"
done
# c5 step after the restore-grid change (bench line + a 20k-step stream)
timeout -k 10 300 python -u bench.py --config c5 --steps 200 --warmup 20 > gpurun_out/r4_c5_bench.log 2>&1 || { tail -5 gpurun_out/r4_c5_bench.log; exit 1; }
tail -1 gpurun_out/r4_c5_bench.log | cut -c1-200
timeout -k 10 400 python -u tools/c5_stream.py stream --steps 20000 --instances 1048576 --ckpt-every 10000 --out gpurun_out/r4_c5_stream_20k.json > gpurun_out/r4_c5_stream_20k.log 2>&1 || { tail -5 gpurun_out/r4_c5_stream_20k.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4_c5_stream_20k.json')); print('c5 stream', d['ms_per_step'], d['replay_seconds'], d['restart_equivalent'])"
