#!/usr/bin/env bash
# On the GPU box: same-box A/B of variants over PT / BDPT / bunny PT / bunny BDPT (512 spp).
#   scripts/gpu_ab4.sh name1 name2 ...   ("default" = the in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/ab_repeat.sh 1 "--mode pt --steps 10 --warmup 3" "$@" && \
scripts/ab_repeat.sh 1 "--mode pt --scene bunny --steps 10 --warmup 3" "$@" && \
scripts/ab_repeat.sh 1 "--mode bdpt --steps 2 --warmup 1" "$@" && \
scripts/ab_repeat.sh 1 "--mode c5 --spp 256 --steps 1 --warmup 1" "$@"
