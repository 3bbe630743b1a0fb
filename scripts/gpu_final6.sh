#!/usr/bin/env bash
# On the GPU box (round 6): the committed evidence for the round's last build.
#   scripts/gpu_final6.sh profile TAG   -> every PMC pass of every BASELINE workload (profile_round.sh)
#   scripts/gpu_final6.sh bench TAG     -> default bench line + its kernel trace, GPU tests, smoke
# Each step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
what=$1; tag=$2
case $what in
  profile)
    bash scripts/profile_round.sh "$tag" pt bdpt c5 c4_ball c4_smooth ;;
  bench)
    timeout -k 10 500 python bench.py > gpurun_out/bench_$tag.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$tag.log; exit 1; }
    tail -c 600 gpurun_out/bench_$tag.log
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/benchkt_$tag -o run --output-format csv -- \
      python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/benchkt_$tag.log 2>&1 || { echo "benchkt failed"; exit 1; }
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
      > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
    tail -2 gpurun_out/${tag}_gpu_tests.log
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
    cat gpurun_out/${tag}_smoke.log ;;
  *) echo "usage: $0 profile|bench TAG"; exit 2 ;;
esac
