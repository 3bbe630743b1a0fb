#!/usr/bin/env bash
# Build oracle/_ref/libref.so: the REAL reference renderer, compiled in place from
# /root/reference (read-only; never copied into the repo) plus oracle/ref_harness.cpp.
# TEST INFRASTRUCTURE ONLY -- output goes to oracle/_ref/ (git-ignored, travels to
# the GPU box as a prebuilt .so).  Recipe follows SURVEY.md §8(c):
#   * g++ -std=gnu++17 -O2 -fpermissive, forced include oracle/absfix.hpp
#     (float abs semantics);
#   * BDPT.cpp:141 binds a non-const reference to a temporary (hard error in g++):
#     it is compiled from a one-token on-the-fly sed of the original file
#     (`auto& lastVertex` -> `auto lastVertex`; PathVertex is a {path*,index}
#     handle so behaviour is unchanged).  No patched copy is written anywhere.
#   * PathTracer.cpp is compiled a second time with the HEAD `break` (:109)
#     removed, as PathTraceIndirect (TPT_MODE_PT_INDIRECT's reference);
#   * main.cpp is not linked (the harness provides the scene presets).
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -d "$REF" ]; then echo "build_ref: $REF not present, skipping"; exit 0; fi
mkdir -p "$OUT/obj"
CXX=${CXX:-g++}
FLAGS="-std=gnu++17 -O2 -fPIC -fpermissive -w -include $HERE/absfix.hpp -I$REF"
SRCS="BVH Material PathTracer Random Renderer SampleHelperFunctions Scene SceneRenderingHelper Sphere Triangle Vector global"
pids=()
for s in $SRCS; do
  $CXX $FLAGS -c "$REF/$s.cpp" -o "$OUT/obj/$s.o" & pids+=($!)
done
sed 's/auto& lastVertex = this->operator\[\](count - 1);/auto lastVertex = this->operator[](count - 1);/' "$REF/BDPT.cpp" \
  | $CXX $FLAGS -x c++ -c - -o "$OUT/obj/BDPT.o" & pids+=($!)
# TPT_MODE_PT_INDIRECT's reference: PathTracer.cpp once more, with the `break` at
# :109 (the end of the HEAD iteration) dropped and the function renamed
# PathTraceIndirect, again through a sed pipe.  Refuse if :109 is not that line.
sed -n '109p' "$REF/PathTracer.cpp" | grep -qx '[[:space:]]*break;[[:space:]]*' \
  || { echo "build_ref: PathTracer.cpp:109 is not the HEAD break" >&2; exit 1; }
sed -e '109s/break;//' -e 's/^Vector3f PathTrace(/Vector3f PathTraceIndirect(/' "$REF/PathTracer.cpp" \
  | $CXX $FLAGS -x c++ -c - -o "$OUT/obj/PathTracerIndirect.o" & pids+=($!)
$CXX $FLAGS -c "$HERE/ref_harness.cpp" -o "$OUT/obj/ref_harness.o" & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
WRAP=_Z19SaveFloatImageToJpgSt6vectorI8Vector3fSaIS0_EEiiNSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEE
$CXX -shared -o "$OUT/libref.so" "$OUT"/obj/*.o -Wl,--wrap=$WRAP -lpthread
echo "build_ref: built $OUT/libref.so"
