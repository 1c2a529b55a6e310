#!/bin/bash
# round-3 session 2 tree: full GPU suite, smoke, bench (headline line), rocprof kernel stats of the bench, TP fused
# all-reduce timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3c
T="python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "r3c/gpu_tests:900:$T" \
  "r3c/smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "r3c/bench:400:python -u bench.py" \
  "r3c/prof:400:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c/prof -o bench -- python bench.py --no-traffic --no-cpu-baseline" \
  "r3c/tp_time:300:python -u tools/tp_fused_time.py"
