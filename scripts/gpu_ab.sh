#!/usr/bin/env bash
# On the GPU box: the -m gpu suite on the in-tree build, then interleaved A/B timings
# (scripts/ab_repeat.sh) of the in-tree build against variants/<names>.
#   scripts/gpu_ab.sh ROUNDS "bench args" [variant ...]   (e.g. scripts/gpu_ab.sh 2 "--mode c5 --spp 256 --steps 1 --warmup 1" base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; args=$2; shift 2
scripts/gpu_run.sh "tests:400:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" || exit 1
grep -E "passed|failed" gpurun_out/tests.log | tail -1
grep -q " failed" gpurun_out/tests.log && exit 1
rm -f gpurun_out/ab.log
timeout -k 10 900 scripts/ab_repeat.sh "$R" "$args" default "$@"
