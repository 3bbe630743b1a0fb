#!/usr/bin/env bash
# Round 5 A/B on the GPU box: shard model + whole-frame BDPT (Standard, bunny 256 spp) and PT
# for each variant (interleaved).   scripts/gpu_ab5.sh name1 name2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 scripts/ab_shard.sh "$@" || exit 1
for i in 1 2; do
  timeout -k 10 300 scripts/ab_repeat.sh 1 "--scene bunny --mode bdpt --spp 256 --steps 2 --warmup 1" default "$@" || exit 1
  timeout -k 10 300 scripts/ab_repeat.sh 1 "--mode bdpt --steps 2 --warmup 1" default "$@" || exit 1
done
