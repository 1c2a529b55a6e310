#!/bin/bash
# last check of the committed tree: GPU suite, smoke, default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/last
T="python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "last/gpu_tests:900:$T" \
  "last/smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "last/bench:400:python -u bench.py --steps 20 --warmup 5"
