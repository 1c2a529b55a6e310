set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 400 --timeout-method thread > gpurun_out/engine_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/engine_trace.py 32 full tools/_lab/liblga_engine_trace.so > gpurun_out/engine_trace.log 2>&1 && \
timeout -k 10 300 python -u tools/engine_bench.py 32 > gpurun_out/engine_bench.log 2>&1
