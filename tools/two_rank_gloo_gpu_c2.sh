# two ranks of bench.py --config c2 on the box's one GPU over gloo (the whole-batch graph path at world 2)
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=2 LOCAL_RANK=0
for r in 0 1; do RANK=$r timeout -k 10 240 python bench.py --config c2 --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/tworank_c2_$r.log 2>&1 & done
wait
