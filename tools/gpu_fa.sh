# prefill flash attention: tests + timing (2 workgroups per CU vs 1 with the longest-first 1-D grid)
set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/fa_tests.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 120 python -u tools/prefill_attn_bench.py > gpurun_out/fa_bench.log 2>&1 || exit 1
LGA_ATTN_PF_SMEM=90000 timeout -k 10 120 python -u tools/prefill_attn_bench.py >> gpurun_out/fa_bench.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/prefill_attn_bench.py >> gpurun_out/fa_bench.log 2>&1 || exit 1
