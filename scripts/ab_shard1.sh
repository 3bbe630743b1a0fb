#!/usr/bin/env bash
# On the GPU box: one stride-N shard (rank 0) per variant, interleaved R rounds (kernel ms).
#   scripts/ab_shard1.sh SCENE SPP N R name1 name2 ...   ("default" = the in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
sc=$1; spp=$2; n=$3; R=$4; shift 4
for i in $(seq 1 $R); do
  for v in "$@"; do
    lib=""; [ "$v" != default ] && lib="TPT_LIB=variants/$v/libtpt.so"
    out=$(env $lib timeout -k 10 120 python scripts/diag/shard_run.py $sc bdpt $spp $n 0 2 2>/dev/null | tail -1) || { echo "$v failed"; exit 1; }
    echo "$v $out"
  done
done
