mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/b_3a.json 2> gpurun_out/b_3a.err || exit 1
KVSEP_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --config 2 > gpurun_out/b_2rank.json 2> gpurun_out/b_2rank.err || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu --roundtrip-gib 0 > gpurun_out/b_1rank_torchrun.json 2> gpurun_out/b_1rank.err || exit 1
