#!/usr/bin/env bash
# On the GPU box: vector-memory pipeline counters (TA / TD / TCP) of the walk-heavy
# kernels, one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md slot limits:
# <= 2 TA, <= 2 TD, <= 4 TCP, <= 2 GRBM per pass).
#   scripts/diag/mem_pipe.sh TAG [c5|bdpt|pt ...]   -> gpurun_out/mp_TAG/
set -eu
tag=$1; shift
work=${*:-c5 bdpt}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/mp_$tag
mkdir -p "$out"
timeout -k 10 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || echo "listing failed (ignored)"
run() {
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -s KILL "$to" "$@" > "$out/$name.log" 2>&1 || { echo "step $name failed rc=$?"; tail -5 "$out/$name.log"; exit 1; }
}
PA=TA_TA_BUSY_sum,TA_FLAT_READ_WAVEFRONTS_sum,TD_TD_BUSY_sum,TD_SPI_STALL_sum,GRBM_GUI_ACTIVE
PB=TCP_TOTAL_CACHE_ACCESSES_sum,TCP_TCC_READ_REQ_sum,TCP_PENDING_STALL_CYCLES_sum,TCP_TCR_TCP_STALL_CYCLES_sum,GRBM_GUI_ACTIVE
for w in $work; do
  case $w in
    pt)   B="python bench.py --mode pt --steps 1 --warmup 0 --spp 256 --no-cpu" ;;
    bdpt) B="python bench.py --mode bdpt --steps 1 --warmup 0 --spp 16 --no-cpu" ;;
    c5)   B="python bench.py --mode c5 --steps 1 --warmup 0 --spp 16 --no-cpu" ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
  run ${w}_pa 120 rocprofv3 --pmc $PA --kernel-trace -d "$out/${w}_pa" -o run --output-format csv -- $B
  run ${w}_pb 120 rocprofv3 --pmc $PB --kernel-trace -d "$out/${w}_pb" -o run --output-format csv -- $B
done
echo "=== done $(date +%T)"
