#!/bin/bash
# BASELINE configs 2 (Llama-2-7B bf16) and 5 (Mixtral-8x7B int4, sparse MoE on one GPU) bench lines + prefill GEMM
# rates at a short prompt (M = 64)
exec bash tools/gpu_session.sh \
  "bench_bf16:400:python -u bench.py --quantize bf16 --steps 100 --no-cpu-baseline" \
  "bench_mixtral:500:python -u bench.py --model Mixtral-8x7B-v0.1 --steps 100 --no-cpu-baseline" \
  "rates64:200:python -u tools/gemm_rates.py 64" \
  "gemm_trace:200:python -u tools/gemm_trace.py tools/_lab/q4f_trace.so"
