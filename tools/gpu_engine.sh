set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 400 --timeout-method thread > gpurun_out/engine_tests.log 2>&1
