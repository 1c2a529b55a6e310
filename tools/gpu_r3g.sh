#!/bin/bash
# round-3 final tree (g): full GPU suite, smoke, bench (headline line), rocprof kernel stats of the bench, GEMM rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3g
T="python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "r3g/gpu_tests:900:$T" \
  "r3g/smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "r3g/bench:400:python -u bench.py" \
  "r3g/prof:400:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3g/prof -o bench -- python bench.py --no-traffic --no-cpu-baseline" \
  "r3g/rates2048:300:python -u tools/gemm_rates.py 2048" \
  "r3g/rates64:300:python -u tools/gemm_rates.py 64"
