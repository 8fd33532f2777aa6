#!/bin/bash
# GPU-box driver: runs each GPU step under its own time limit and stops at
# the first fault / abort / timeout (exit status other than 0 or 1).
# usage: scripts/gpu_run.sh "<name>:<seconds>:<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"
  secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: [$name] ended with rc=$rc"
    exit $rc
  fi
done
