#!/usr/bin/env bash
# On the GPU box: kernel-trace stats per variant for a bench workload (per-kernel mean ms).
#   scripts/kt_ab.sh TAG "bench args" variant...   ("default" = in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; args=$2; shift 2
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib="$PWD/variants/$v/libtpt.so"
  TPT_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${tag}_$v -o run \
      --output-format csv -- python bench.py $args --no-cpu > gpurun_out/kt_${tag}_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  python3 - "$v" "gpurun_out/kt_${tag}_$v/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[2])):
    if r["Name"].startswith("tpt_") or "tpt_" in r["Name"][:30]:
        print(sys.argv[1], r["Name"].split("(")[0][-40:], r["Calls"], "%.3f ms avg" % (float(r["AverageNs"]) / 1e6),
              "%.1f ms total" % (float(r["TotalDurationNs"]) / 1e6))
PY
done
