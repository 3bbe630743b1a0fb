#!/usr/bin/env bash
# A/B builds: variants/<name>/libtpt.so = libtpt.so with extra -D flags on the kernel and scene-build TUs.
#   scripts/build_variant.sh nodefer -DTPT_LEAF_DEFER=0
# Load one with TPT_LIB=variants/<name>/libtpt.so (bench.py, tests).  Profiling only.
set -eu
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/toypathtracer-games101-assignment7_amd
out=$root/variants/$name
mkdir -p "$out"
make -s -C "$pkg" build/tpt_multi.o build/scene_api.o build/film.o
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-unused-function "$@" -x c++ -c \
    -o "$out/tpt_scene_build.o" "$pkg/csrc/tpt_scene_build.cpp"
trk="-mllvm -amdgpu-use-amdgpu-trackers=1"
[ "${TRACKERS:-1}" = 0 ] && trk=""  # TRACKERS=0: without the AMDGPU trackers (the Makefile's default has them)
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-unused-function --offload-arch=gfx950 \
    -munsafe-fp-atomics -fno-slp-vectorize $trk "$@" -c -o "$out/tpt_capi.o" "$pkg/csrc/tpt_capi.hip"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-unused-function --offload-arch=gfx950 \
    -munsafe-fp-atomics -fno-slp-vectorize "$@" -c -o "$out/tpt_conn2.o" "$pkg/csrc/tpt_conn2.hip"  # no trackers (Makefile)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out/libtpt.so" "$out/tpt_capi.o" "$out/tpt_conn2.o" \
    "$out/tpt_scene_build.o" "$pkg/build/tpt_multi.o" "$pkg/build/scene_api.o" "$pkg/build/film.o" -ldl
echo "built $out/libtpt.so ($*)"
