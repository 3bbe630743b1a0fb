#!/usr/bin/env bash
# On the GPU box: kernel trace of one stride-N shard, per-wavefront timeline.
#   [TPT_LIB=...] scripts/diag/shard_trace1.sh SCENE MODE SPP N TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
sc=$1; mo=$2; spp=$3; n=$4; tag=$5
d=gpurun_out/st1_${tag}_${sc}_${n}
timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python scripts/diag/shard_run.py $sc $mo $spp $n 0 2 > $d.log 2>&1 || exit 1
f=$(find $d -name '*kernel_trace.csv' | head -1)
echo "== $tag $sc $mo spp $spp N=$n"; grep kernel_ms $d.log
python scripts/diag/wf_timeline.py "$f" 2
