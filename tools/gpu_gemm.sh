# fused prefill GEMM: tests (ping-pong default) + rates, ping-pong vs one-barrier loop
set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_fused_tests.log 2>&1; rc=$?; ok $rc || exit $rc
for m in 2048 512 64; do
  timeout -k 10 200 python -u tools/gemm_rates.py $m lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so q4f,q4f_bf16w,torch_mm,q4f_swiglu/2 > gpurun_out/gemm_rates_m$m.log 2>&1 || exit 1

done
