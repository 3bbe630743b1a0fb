#!/usr/bin/env bash
# On the GPU box: the rocprofv3 evidence behind bench.py's numbers for this build.
#   scripts/profile_round.sh TAG      -> gpurun_out/prof_TAG/{pt,bdpt}_{kt,fetch,write}/
# Kernel-trace --stats of the default PT bench and of the BDPT bench (one frame
# each), then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md
# §HBM/rocprofv3: TCC slots do not hold both).  Each step has its own time limit and
# the script stops at the first failure.
set -eu
tag=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
PT="python bench.py --mode pt --steps 1 --warmup 1 --no-cpu"
BD="python bench.py --mode bdpt --steps 1 --warmup 0 --no-cpu"
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1 || { echo "step $name failed rc=$?"; tail -5 "$out/$name.log"; exit 1; }
}
run pt_kt 180 rocprofv3 --kernel-trace --stats -d "$out/pt_kt" -o run --output-format csv -- $PT
run bdpt_kt 240 rocprofv3 --kernel-trace --stats -d "$out/bdpt_kt" -o run --output-format csv -- $BD
run pt_fetch 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/pt_fetch" -o run --output-format csv -- $PT
run pt_write 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/pt_write" -o run --output-format csv -- $PT
run bdpt_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/bdpt_fetch" -o run --output-format csv -- $BD
run bdpt_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/bdpt_write" -o run --output-format csv -- $BD
run pt_sq 180 rocprofv3 --pmc SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY,SQ_WAVES --kernel-trace -d "$out/pt_sq" -o run --output-format csv -- $PT
echo "=== done"
