# fused prefill GEMM: tests (both tile shapes) + rates
set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_fused_tests.log 2>&1; rc=$?; ok $rc || exit $rc
LGA_Q4F_BM=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_fused_tests256.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 200 python -u tools/gemm_rates.py 2048 > gpurun_out/gemm_rates128.log 2>&1 || exit 1
LGA_Q4F_BM=256 timeout -k 10 200 python -u tools/gemm_rates.py 2048 > gpurun_out/gemm_rates256.log 2>&1 || exit 1
