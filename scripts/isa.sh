#!/usr/bin/env bash
# Device assembly of the kernel TU (with line tables) + spill counts per kernel.  (The
# walk-group scenes' connect kernel is in csrc/tpt_conn2.hip, built without the trackers:
# run with TRACKERS=0 and -DTPT_TU_CONN2=1 on that file for it.)
#   scripts/isa.sh OUT.s [extra hipcc flags...]
set -eu
out=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-unused-function --offload-arch=gfx950 \
  -munsafe-fp-atomics -fno-slp-vectorize -mllvm -amdgpu-use-amdgpu-trackers=1 --cuda-device-only -gline-tables-only -S "$@" -o "$out" \
  "$root/toypathtracer-games101-assignment7_amd/csrc/tpt_capi.hip" 2>&1 | grep -v hip-link || true
python3 "$root/scripts/isa_spills.py" "$out" pt_kernelILi1ELb0ELi8 bdpt_gen bdpt_conn
