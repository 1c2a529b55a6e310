#!/bin/bash
# all-reduce flag protocol without cache maintenance: all-reduce / fused GEMV bit-exact tests at 2/4/8 ranks, the
# late-peer tests, TP=2 graph decode, then the per-call timing
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "t_comm:900:$T tests/test_gpu_tp.py -k 'bit_exact or late_peer or tp2'" \
  "tp_time:300:python -u tools/tp_fused_time.py"
