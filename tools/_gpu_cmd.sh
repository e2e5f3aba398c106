mkdir -p gpurun_out
true && \
BSLS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/bench2_gloo.log 2>&1 && \
timeout -k 10 600 python -u tools/shard_scaling.py --c5 --worlds 8 4 2 1 > gpurun_out/ss_c5.log 2>&1
