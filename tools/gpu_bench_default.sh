mkdir -p gpurun_out
timeout -k 10 120 python tools/probe_gelu_kind.py > gpurun_out/gelu_kind.txt 2>&1; cat gpurun_out/gelu_kind.txt
timeout -k 10 400 python bench.py > gpurun_out/b_c3_default.log 2>&1 || { tail -5 gpurun_out/b_c3_default.log; exit 1; }
grep '^{' gpurun_out/b_c3_default.log
