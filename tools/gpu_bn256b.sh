#!/bin/bash
# A/B after the fence-free split-K: every shape on 256 x 256 tiles (proj / down then split K in two) vs the planner
exec bash tools/gpu_session.sh \
  "rates_plan:200:python -u tools/gemm_rates.py 2048 '' q4f,q4f_swiglu/2" \
  "rates_256:200:LGA_Q4F_BN=256 python -u tools/gemm_rates.py 2048 '' q4f,q4f_swiglu/2" \
  "rates_plan2:200:python -u tools/gemm_rates.py 2048 '' q4f,q4f_swiglu/2"
