#!/bin/bash
# Runs named GPU steps, each under its own time limit; stops at the first fault/timeout/crash.
# usage: tools/gpu_session.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
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
