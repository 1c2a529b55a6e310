#!/bin/bash
# argmax at 4 waves: its tests, the generate / graph tests, the bench and a rocprof pass for the per-step kernel time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "t_argmax:400:$T tests/test_gpu_kernels.py -k 'argmax or embed'" \
  "t_model:600:$T tests/test_gpu_model.py" \
  "bench:300:python -u bench.py --no-cpu-baseline" \
  "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/argmax_prof -o bench -- python bench.py --no-traffic --no-cpu-baseline"
