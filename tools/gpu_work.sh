# engine + fused prefill GEMM: tests, rates, engine trace / A-B (one GPU call); a test FAILURE (exit 1) does not
# stop the call, anything else (fault, abort, time limit) does
set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_fused_tests.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 200 python -u tools/gemm_rates.py 2048 > gpurun_out/gemm_rates.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 400 --timeout-method thread > gpurun_out/engine_tests.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 300 python -u tools/engine_trace.py 32 full tools/_lab/liblga_engine_trace.so > gpurun_out/engine_trace.log 2>&1 && \
timeout -k 10 300 python -u tools/engine_bench.py 32 > gpurun_out/engine_bench.log 2>&1
