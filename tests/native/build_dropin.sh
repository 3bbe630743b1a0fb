#!/usr/bin/env bash
# Drop-in check of the C++ caller surface: compile the reference's OWN, unmodified
# main.cpp (/root/reference/main.cpp, read through a pipe; nothing is copied) against
# include/tpt_scene_api.hpp and link it to libtpt.so.  The reference's headers
# (Renderer.hpp, Scene.hpp, Triangle.hpp, ...) are each mapped to the drop-in header
# by a one-line include in tests/native/build/shim/.  Output:
#   tests/native/build/ref_main_tpt   (git-ignored; travels to the GPU box, where
#                                      tests/test_gpu_parity.py::test_reference_main_drop_in runs it)
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
PKG="$ROOT/toypathtracer-games101-assignment7_amd"
OUT="$HERE/build"
if [ ! -f "$REF/main.cpp" ]; then echo "build_dropin: $REF/main.cpp not present, skipping"; exit 0; fi
mkdir -p "$OUT/shim"
for h in global Renderer Scene Triangle Sphere Vector SceneRenderingHelper SampleHelperFunctions BDPT Material; do
  echo '#include "tpt_scene_api.hpp"' > "$OUT/shim/$h.hpp"
done
# from stdin and inside $OUT, so the quoted includes resolve to the shims, not to $REF
( cd "$OUT" && ${CXX:-g++} -std=c++17 -O2 -I"$OUT/shim" -I"$ROOT/include" -x c++ - < "$REF/main.cpp" \
    -L"$PKG" -ltpt -Wl,-rpath,'$ORIGIN/../../../toypathtracer-games101-assignment7_amd' -o "$OUT/ref_main_tpt" )
echo "build_dropin: built $OUT/ref_main_tpt"
