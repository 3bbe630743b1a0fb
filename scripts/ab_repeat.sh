#!/usr/bin/env bash
# On the GPU box: interleaved A/B timing (ABAB...) of variants, R rounds.
#   scripts/ab_repeat.sh R "bench args" name1 name2 ...   (name "default" = the in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; args=$2; shift 2
for i in $(seq 1 $R); do
  for v in "$@"; do
    lib=""; [ "$v" != default ] && lib="TPT_LIB=variants/$v/libtpt.so"
    out=$(env $lib timeout -k 10 120 python bench.py $args --no-cpu 2>/dev/null | tail -1) || { echo "$v failed"; exit 1; }
    echo "$v $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")" | tee -a gpurun_out/ab.log
  done
done
