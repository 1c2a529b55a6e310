# fused prefill GEMM: tests, rates (product library), then the bench line
set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_fused.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_fused_tests.log 2>&1; rc=$?; ok $rc || exit $rc
for m in 2048 64; do
  timeout -k 10 200 python -u tools/gemm_rates.py $m lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so q4f,q4f_bf16w,q4f_swiglu/2 > gpurun_out/gemm_rates_m$m.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_gemm.log 2>&1
