#!/usr/bin/env bash
# On the GPU box: kernel traces of the full frame and one 1/8 shard.  scripts/diag/shard_trace.sh SCENE MODE SPP
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
sc=$1; mo=$2; spp=$3
for n in 1 8; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/st_${sc}_${mo}_$n -o run --output-format csv -- python scripts/diag/shard_run.py $sc $mo $spp $n 0 2 > gpurun_out/st_${sc}_${mo}_$n.log 2>&1 || exit 1
  f=$(find gpurun_out/st_${sc}_${mo}_$n -name '*kernel_trace.csv' | head -1)
  echo "== $sc $mo spp $spp N=$n"; grep kernel_ms gpurun_out/st_${sc}_${mo}_$n.log
  python scripts/diag/trace_timeline.py "$f"
done
