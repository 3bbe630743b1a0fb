#!/usr/bin/env bash
# On the GPU box, one call: this build's profiles (scripts/profile_round.sh), the default
# bench line and its kernel trace (scripts/gpu_bench_round.sh), and the PT per-wave
# timing of a 1/8 shard (diagnostics variant).   scripts/gpu_round3.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
scripts/profile_round.sh "$tag" pt bdpt c5 c4_ball c4_smooth > gpurun_out/profile_$tag.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/profile_$tag.log; exit 1; }
echo "profiles done"
scripts/gpu_bench_round.sh "$tag" || { echo "bench failed"; exit 1; }
echo "bench done"
if [ -f variants/wt/libtpt.so ]; then
  TPT_LIB=variants/wt/libtpt.so timeout -k 10 120 python -u scripts/diag/pt_wavetime.py > gpurun_out/wt_$tag.log 2>&1 || echo "wavetime failed"
fi
echo "all done"
