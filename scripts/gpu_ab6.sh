#!/usr/bin/env bash
# On the GPU box (round 6): frame pins of a variant, then interleaved timing against the
# in-tree build.   scripts/gpu_ab6.sh "pytest -k expr" R "bench args" name1 name2 ...
# Each step has its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
sel=$1; R=$2; args=$3; shift 3
for v in "$@"; do
  [ "$v" = default ] && continue
  [ -z "$sel" ] && continue
  echo "== pins $v: $sel"
  TPT_LIB=variants/$v/libtpt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py \
    -m gpu -x -q --timeout 240 --timeout-method thread -k "$sel" > gpurun_out/pins_$v.log 2>&1 || { echo "pins $v FAILED"; tail -30 gpurun_out/pins_$v.log; exit 1; }
  tail -1 gpurun_out/pins_$v.log
done
for i in $(seq 1 $R); do
  for v in "$@"; do
    lib=""; [ "$v" != default ] && lib="TPT_LIB=variants/$v/libtpt.so"
    out=$(env $lib timeout -k 10 300 python bench.py $args --no-cpu 2>/dev/null | tail -1) || { echo "$v failed"; exit 1; }
    echo "$v $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('shard_model'); print(d.get('ms_per_step'), d.get('kernel_ms_per_step'), {k: (v.get('full_kernel_ms'), [(n, v[n].get('eff_kernel'), max(v[n]['kernel_ms'])) for n in ('n2', 'n4', 'n8') if n in v]) for k, v in (s or {}).items() if isinstance(v, dict)})")" | tee -a gpurun_out/ab6.log
  done
done
