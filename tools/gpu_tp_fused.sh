#!/bin/bash
# fused row-parallel GEMV + all-reduce: parity tests, then per-call timing vs the two-launch form
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "t_fused:400:$T tests/test_gpu_tp.py -k fused_gemv" \
  "tp_time:300:python -u tools/tp_fused_time.py"
