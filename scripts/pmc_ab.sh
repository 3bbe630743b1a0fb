#!/usr/bin/env bash
# On the GPU box: one PMC pass per variant for a bench workload.
#   scripts/pmc_ab.sh TAG COUNTERS "bench args" variant...   ("default" = in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; ctr=$2; args=$3; shift 3
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib="$PWD/variants/$v/libtpt.so"
  TPT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc_${tag}_$v -o run \
      --output-format csv -- python bench.py $args --no-cpu > gpurun_out/pmc_${tag}_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/pmc_${tag}_$v/run_counter_collection.csv | sed "s/^/$v /"
done
