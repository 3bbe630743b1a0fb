#!/usr/bin/env bash
# Per-kernel VGPRs / scratch / occupancy / LDS of the kernel TU (make resource-usage), one line per kernel.
#   scripts/ru.sh [name-substring]
cd "$(dirname "$0")/../toypathtracer-games101-assignment7_amd"
make -s resource-usage 2>&1 | python3 -c "
import re, sys
cur = None; rows = {}
for l in sys.stdin:
    m = re.search(r'Function Name: (\S+)', l)
    if m: cur = m.group(1); rows[cur] = {}; continue
    for k in ('VGPRs', 'ScratchSize \[bytes/lane\]', 'Occupancy \[waves/SIMD\]', 'LDS Size \[bytes/block\]'):
        m = re.search(k + r': (\d+)', l)
        if m and cur: rows[cur][k.split()[0].split('\\\\')[0]] = int(m.group(1))
pat = sys.argv[1] if len(sys.argv) > 1 else ''
for f, r in rows.items():
    if pat in f: print('%-70s %s' % (f[:70], ' '.join('%s=%s' % kv for kv in r.items())))
" "$@"
