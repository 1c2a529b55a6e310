#!/bin/bash
# rehearsal of the driver's multi-GPU bench invocation on a one-GPU box: 2 and 4 ranks on cuda:0 (gloo for the
# host collectives, xGMI kernel for the decode all-reduces); checks that bench.py's TP path runs end to end and
# prints its JSON line (the numbers share one device: not a scaling measurement)
set -o pipefail
mkdir -p gpurun_out
export LGA_ONE_DEVICE=1 LGA_DIST_BACKEND=gloo OMP_NUM_THREADS=2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 16 --warmup 8 --no-cpu-baseline > gpurun_out/bench_tp2.log 2>&1 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 4 --steps 16 --warmup 8 --no-cpu-baseline > gpurun_out/bench_tp4.log 2>&1 || exit 1
tail -1 gpurun_out/bench_tp2.log; tail -1 gpurun_out/bench_tp4.log
