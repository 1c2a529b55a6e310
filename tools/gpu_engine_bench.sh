set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/engine_bench.py 32 > gpurun_out/engine_bench.log 2>&1
