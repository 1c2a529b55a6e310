#!/bin/bash
# 256 x 256 fc tiles on by the planner: fused GEMM tests, the 7B-geometry / model tests that prefill 2048 tokens,
# rates, bench
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "t_gemm:400:$T tests/test_gpu_gemm_fused.py" \
  "t_geom:700:$T tests/test_gpu_geometry.py tests/test_gpu_model.py" \
  "rates:200:python -u tools/gemm_rates.py 2048" \
  "bench:300:python -u bench.py --no-cpu-baseline"
