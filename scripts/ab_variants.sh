#!/usr/bin/env bash
# On the GPU box: time bench.py workloads for each variants/<name>/libtpt.so (TPT_LIB)
# next to the default build.   scripts/ab_variants.sh "mode args" name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
args=$1; shift
for v in default "$@"; do
  lib=""; [ "$v" != default ] && lib="TPT_LIB=variants/$v/libtpt.so"
  out=$(env $lib timeout -k 10 120 python bench.py $args --no-cpu 2>/dev/null | tail -1) || { echo "$v failed"; exit 1; }
  echo "$v $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms/step', d['kernel_ms_per_step'], 'kernel ms')")" | tee -a gpurun_out/ab.log
done
