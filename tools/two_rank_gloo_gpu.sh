# two ranks of bench.py on the box's one GPU over gloo (rehearses the multi-rank bench path on GPU tensors;
# the RCCL transport itself needs one GPU per rank)
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=2 LOCAL_RANK=0
for r in 0 1; do RANK=$r timeout -k 10 240 python bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/tworank_$r.log 2>&1 & done
wait
tail -3 gpurun_out/tworank_0.log; tail -3 gpurun_out/tworank_1.log
