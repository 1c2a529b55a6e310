# final-tree measurement: GPU suite, smoke, default bench line, rocprof kernel stats of the bench (decode breakdown on CPU afterwards)
set -o pipefail
mkdir -p gpurun_out/final
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/final/gpu_tests.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o bench -- python bench.py --no-traffic --no-cpu-baseline > gpurun_out/final/prof.log 2>&1
