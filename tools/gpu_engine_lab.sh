# lab: the persistent decode engine (tools/lab/engine) — its parity tests and the A/B against the per-op graph
set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tools/lab/engine/test_engine.py -x -q -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/engine_lab_tests.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 300 python -u tools/lab/engine/engine_bench.py 32 > gpurun_out/engine_lab_bench.log 2>&1
