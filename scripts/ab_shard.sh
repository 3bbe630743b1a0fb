#!/usr/bin/env bash
# On the GPU box: the shard model (bench.py --shard-only) for each variants/<name>/libtpt.so
# next to the default build.   scripts/ab_shard.sh name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in default "$@"; do
  lib=""; [ "$v" != default ] && lib="TPT_LIB=variants/$v/libtpt.so"
  env $lib timeout -k 10 300 python bench.py --shard-only > gpurun_out/shard_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/shard_$v.log; exit 1; }
  tail -1 gpurun_out/shard_$v.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())['shard_model']
print('$v', ' '.join('%s full %.1f ms eff %s' % (k, d[k]['full_kernel_ms'], '/'.join('%.3f' % d[k]['n%d' % n]['eff_kernel'] for n in d['ns'])) for k in ('pt', 'bdpt', 'c5')))" | tee -a gpurun_out/ab.log
done
