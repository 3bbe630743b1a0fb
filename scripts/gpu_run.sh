#!/usr/bin/env bash
# Run on the GPU box via gpurun.  Steps stop at the first fault/timeout/abort
# (exit >= 124 or a signal); an ordinary test failure (exit 1) lets later steps run.
# usage: scripts/gpu_run.sh "step-name:timeout:command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name (timeout $to s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
done
