#!/usr/bin/env bash
# On the GPU box: per-kernel BDPT times (serial-stream variant) + PTI compaction A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
TPT_LIB=variants/serial/libtpt.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ser -o run --output-format csv -- python bench.py --mode bdpt --steps 1 --warmup 0 --spp 32 --no-cpu > gpurun_out/ser.log 2>&1 && \
scripts/ab_repeat.sh 2 "--mode pti --steps 2 --warmup 1" default ptic
