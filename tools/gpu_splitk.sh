#!/bin/bash
# fence-free split-K (write-through slabs): fused GEMM tests, short-prompt rates, short-prompt model tests
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "t_gemm:400:$T tests/test_gpu_gemm_fused.py" \
  "rates64:300:python -u tools/gemm_rates.py 64" \
  "rates128:300:python -u tools/gemm_rates.py 128" \
  "t_model:600:$T tests/test_gpu_model.py"
