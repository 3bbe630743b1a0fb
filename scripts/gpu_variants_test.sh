#!/usr/bin/env bash
# Run one pytest selection against several library variants ("default" = in-tree build).
#   scripts/gpu_variants_test.sh "pytest -k expr" name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
sel=$1; shift
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib="TPT_LIB=variants/$v/libtpt.so"
  env $lib timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "$sel" > gpurun_out/vt_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/vt_$v.log)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
