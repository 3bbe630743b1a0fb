#!/usr/bin/env bash
# On the GPU box: the rocprofv3 evidence behind bench.py's numbers for this build.
#   scripts/profile_round.sh TAG [pt|bdpt|c5|pti|c4_ball|c4_smooth ...]   -> gpurun_out/prof_TAG/<workload>_<pass>/
# Per workload: a kernel-trace --stats pass, then the PMC passes (one rocprofv3 run
# each, MI355X_MICROARCH.md §rocprofv3 PMC slots: <= 8 SQ, <= 4 TCC of which
# FETCH_SIZE takes 3 and WRITE_SIZE 2, <= 2 GRBM):
#   valu1  SQ_INSTS_VALU + the f32 / f64 add, mul, fma and f32 transcendental classes
#   valu2  f64 transcendental, int32, int64, cvt classes, VALU / wave / busy cycles,
#          GRBM_GUI_ACTIVE (the clock the run held)
#   misc   SALU / LDS / VMEM / SMEM instruction counts and the wait buckets
#   fetch  FETCH_SIZE ; write  WRITE_SIZE
#   lane   SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU: VALU lane utilisation (round 6;
#          counter_defs.yaml's VALUUtilization = THREAD_CYCLES / (64 x ACTIVE_INST_VALU))
# PASSES="kt lane ..." runs a subset (default: all); NOCOST=1 skips valu_cost.
# and, once per call, scripts/valu_cost (cycles per wave-instruction of each class).
# Each step has its own time limit; the script stops at the first failure.
set -eu
tag=$1; shift
work=${*:-pt bdpt}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1 || { echo "step $name failed rc=$?"; tail -5 "$out/$name.log"; exit 1; }
}
P1=SQ_INSTS_VALU,SQ_INSTS_VALU_ADD_F32,SQ_INSTS_VALU_MUL_F32,SQ_INSTS_VALU_FMA_F32,SQ_INSTS_VALU_TRANS_F32,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64
P2=SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_INT32,SQ_INSTS_VALU_INT64,SQ_INSTS_VALU_CVT,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE,GRBM_COUNT
P4=SQ_THREAD_CYCLES_VALU,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_WAVES
P3=SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_SMEM,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_WAVES
passes=${PASSES:-kt valu1 valu2 misc fetch write lane}
prun() {  # pass workload-name timeout args...: run() when the pass is selected
  local p=$1; shift
  case " $passes " in *" $p "*) run "$@" ;; esac
  return 0
}
[ -n "${NOCOST:-}" ] || run valu_cost 120 scripts/valu_cost
for w in $work; do
  case $w in
    pt)   B="python bench.py --mode pt --steps 1 --warmup 1 --no-cpu" ;;
    bdpt) B="python bench.py --mode bdpt --steps 1 --warmup 0 --spp 32 --no-cpu" ;;
    c5)   B="python bench.py --mode c5 --steps 1 --warmup 0 --spp 32 --no-cpu" ;;
    pti)  B="python bench.py --mode pti --steps 1 --warmup 0 --spp 64 --no-cpu" ;;
    c4_ball)   B="python bench.py --mode c4_ball --steps 1 --warmup 0 --spp 1024 --no-cpu" ;;
    c4_smooth) B="python bench.py --mode c4_smooth --steps 1 --warmup 0 --spp 1024 --no-cpu" ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
  prun kt ${w}_kt 240 rocprofv3 --kernel-trace --stats -d "$out/${w}_kt" -o run --output-format csv -- $B
  prun valu1 ${w}_valu1 180 rocprofv3 --pmc $P1 --kernel-trace -d "$out/${w}_valu1" -o run --output-format csv -- $B
  prun valu2 ${w}_valu2 180 rocprofv3 --pmc $P2 --kernel-trace -d "$out/${w}_valu2" -o run --output-format csv -- $B
  prun misc ${w}_misc 180 rocprofv3 --pmc $P3 --kernel-trace -d "$out/${w}_misc" -o run --output-format csv -- $B
  prun fetch ${w}_fetch 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/${w}_fetch" -o run --output-format csv -- $B
  prun write ${w}_write 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/${w}_write" -o run --output-format csv -- $B
  prun lane ${w}_lane 180 rocprofv3 --pmc $P4 --kernel-trace -d "$out/${w}_lane" -o run --output-format csv -- $B
done
echo "=== done $(date +%T)"
