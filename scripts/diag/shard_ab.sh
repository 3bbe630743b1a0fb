#!/usr/bin/env bash
# On the GPU box: kernel ms of one stride-N shard per variant, interleaved R rounds.
#   scripts/diag/shard_ab.sh R SCENE MODE SPP N variant...  ("default" = in-tree build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
R=$1; scene=$2; mode=$3; spp=$4; n=$5; shift 5
for i in $(seq 1 $R); do
  for v in "$@"; do
    lib=""; [ "$v" != default ] && lib="TPT_LIB=variants/$v/libtpt.so"
    out=$(env $lib timeout -k 10 120 python scripts/diag/shard_run.py $scene $mode $spp $n 0 3 2>/dev/null | tail -1) || { echo "$v failed"; exit 1; }
    echo "$v $scene $mode $spp 1/$n $out" | tee -a gpurun_out/shard_ab.log
  done
done
