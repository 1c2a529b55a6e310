#!/bin/bash
# The one GPU session script: named steps, each under its own time limit, stopping at the first fault / timeout /
# crash (a test FAILURE, rc 1, does not stop the session). Logs land in gpurun_out/<name>.log.
#
# usage: tools/gpu_session.sh STEP...
#   STEP = "name:seconds:command"            one step
#        | "@preset:tag"                     a preset expanded into steps named tag/...
# presets:
#   @tests:TAG   the whole -m gpu suite                @smoke:TAG  __graft_entry__.smoke()
#   @bench:TAG   bench.py (driver defaults)            @prof:TAG   rocprofv3 kernel trace + stats of bench.py
#   @last:TAG    tests + smoke + bench + prof: the last check of a committed tree
#   @tp:TAG      the driver's multi-GPU bench invocation rehearsed with 2 ranks on the one GPU (LGA_ONE_DEVICE=1, gloo
#                host collectives, xGMI-kernel decode all-reduces): the TP path end to end, NOT a scaling number
# e.g. /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_session.sh @last:r04z'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider"
PROF="cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv"
expand() {  # preset:tag -> step specs, one per line
  local p="${1%%:*}" tag="${1#*:}"
  case "$p" in
    @tests) echo "$tag/gpu_tests:1200:$T" ;;
    @smoke) echo "$tag/smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" ;;
    @bench) echo "$tag/bench:400:python -u bench.py" ;;
    @prof) echo "$tag/prof:400:$PROF -d gpurun_out/$tag/prof -o bench -- python bench.py --no-traffic --no-cpu-baseline" ;;
    @last) expand "@tests:$tag"; expand "@smoke:$tag"; expand "@bench:$tag"; expand "@prof:$tag" ;;
    @tp) echo "$tag/bench_tp2:400:LGA_ONE_DEVICE=1 LGA_DIST_BACKEND=gloo OMP_NUM_THREADS=2 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 16 --warmup 8 --no-cpu-baseline" ;;
    *) echo "unknown preset $p" >&2; return 1 ;;
  esac
}
steps=()
for a in "$@"; do
  if [[ "$a" == @* ]]; then
    expand "$a" > /dev/null || exit 2
    while IFS= read -r s; do steps+=("$s"); done < <(expand "$a")
  else
    steps+=("$a")
  fi
done
for spec in "${steps[@]}"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  mkdir -p "$(dirname "gpurun_out/$name.log")"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - start ))s"
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1) ;;             # success or ordinary test failures: keep going
    *) echo "stopping after $name (rc=$rc)"; exit $rc ;;
  esac
done
