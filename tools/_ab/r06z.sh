bash tools/gpu_session.sh \
 "r06z/tp2_tagged:400:LGA_ONE_DEVICE=1 LGA_AR_PROTOCOL=tagged LGA_DIST_BACKEND=gloo OMP_NUM_THREADS=2 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29563 bench.py --gpus 2 --steps 16 --warmup 8 --no-cpu-baseline --no-traffic" \
 "r06z/tp4_tagged:400:LGA_ONE_DEVICE=1 LGA_AR_PROTOCOL=tagged LGA_DIST_BACKEND=gloo OMP_NUM_THREADS=2 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29564 bench.py --gpus 4 --steps 16 --warmup 8 --no-cpu-baseline --no-traffic"
