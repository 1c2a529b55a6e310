#!/bin/bash
# A/B: 256 x 256 fused-GEMM tiles (64 x 128 outputs per wave) vs 256 x 128 at M = 2048; tests with the big tile on
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "t_bn256:400:LGA_Q4F_BN256=1 $T tests/test_gpu_gemm_fused.py" \
  "rates_128:200:python -u tools/gemm_rates.py 2048" \
  "rates_256:200:LGA_Q4F_BN256=1 python -u tools/gemm_rates.py 2048" \
  "rates_128b:200:python -u tools/gemm_rates.py 2048"
