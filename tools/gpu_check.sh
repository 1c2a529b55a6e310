set -o pipefail
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_tp.py -x -v --timeout 600 --timeout-method thread -k "xgmi_allreduce or tp8" > gpurun_out/tp.log 2>&1
