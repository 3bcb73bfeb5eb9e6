# N=2 rehearsal of the decomposed bench on the one-GPU box (both ranks on device 0)
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_n2_decomposed.log 2>&1
echo "rc=$?"; tail -c 3000 gpurun_out/bench_n2_decomposed.log
