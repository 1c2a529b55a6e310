# fused GEMM A/B (setprio on/off, tile shapes), then the TP tests (8-rank xGMI, late peer) and smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/gemm_rates.py 2048 lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so q4f,q4f_bf16w,blaslt,q4f_swiglu/2 > gpurun_out/gr_prio.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/gemm_rates.py 2048 tools/_lab/liblga_q4f_noprio.so q4f,q4f_bf16w,blaslt,q4f_swiglu/2 > gpurun_out/gr_noprio.log 2>&1 || exit 1
LGA_Q4F_BM=128 timeout -k 10 200 python -u tools/gemm_rates.py 2048 lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so q4f,q4f_bf16w,q4f_swiglu/2 > gpurun_out/gr_prio128.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_tp.py -x -v --timeout 600 --timeout-method thread -k "xgmi_allreduce or tp8" > gpurun_out/tp.log 2>&1
