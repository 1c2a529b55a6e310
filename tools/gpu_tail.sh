#!/bin/bash
# fused GEMM tail-round split: tests, per-shape rates with / without it, the bench's cold / warm prefill
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "t_gemm:400:$T tests/test_gpu_gemm_fused.py" \
  "rates_tail:200:python -u tools/gemm_rates.py 2048" \
  "rates_notail:200:LGA_Q4F_NO_TAIL_SPLIT=1 python -u tools/gemm_rates.py 2048" \
  "bench:300:python -u bench.py --no-cpu-baseline"
