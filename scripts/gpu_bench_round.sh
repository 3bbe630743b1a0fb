#!/usr/bin/env bash
# On the GPU box: the default bench line (as the driver runs it) and a kernel-trace of
# the same command.   scripts/gpu_bench_round.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
tag=$1
timeout -k 10 400 python bench.py > gpurun_out/bench_$tag.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/benchkt_$tag -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/benchkt_$tag.log 2>&1
