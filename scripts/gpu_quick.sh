#!/usr/bin/env bash
# On the GPU box: GPU parity suite + PT / BDPT / c5 bench lines (no CPU legs).
#   scripts/gpu_quick.sh [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K=${1:+-k "$1"}
scripts/gpu_run.sh "tests:600:python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread $K" \
  "pt:120:python bench.py --mode pt --steps 20 --warmup 5 --no-cpu" \
  "bdpt:120:python bench.py --mode bdpt --steps 3 --warmup 1 --no-cpu" \
  "c5:180:python bench.py --mode c5 --spp 512 --steps 1 --warmup 0 --no-cpu"
grep -E "passed|failed" gpurun_out/tests.log | tail -1
for f in pt bdpt c5; do python -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], 'Msamples/s', d['ms_per_step'], 'ms/step', 'valu frac', r.get('frac'))" 2>/dev/null || echo "$f: no line"; done
