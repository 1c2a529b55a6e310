# prefill flash attention: tests + timing (causal, and every row seeing all keys)
set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "attention or prefill" --timeout 120 --timeout-method thread > gpurun_out/fa_tests.log 2>&1; rc=$?; ok $rc || exit $rc
for i in 1 2; do
timeout -k 10 120 python -u tools/prefill_attn_bench.py > gpurun_out/fa_bench_$i.log 2>&1 || exit 1
ATT_FULL=1 timeout -k 10 120 python -u tools/prefill_attn_bench.py >> gpurun_out/fa_bench_$i.log 2>&1 || exit 1
done
