"""Compare the device ISA of two builds kernel by kernel (labels normalised).
    python scripts/isa_cmp.py OLD.s NEW.s   (OLD/NEW from: hipcc ... --cuda-device-only -S)"""
import re, sys
def kernels(path):
    out={}; cur=None
    for l in open(path):
        m=re.match(r'^(_Z\w+):', l)
        if m: cur=m.group(1); out[cur]=[]; continue
        if cur is None: continue
        s=l.strip()
        if s.startswith('s_endpgm'): out[cur].append(s); cur=None; continue
        if not s or s.startswith(('.',';','//')) or re.match(r'^\.?L\w+:', s): continue
        out[cur].append(re.sub(r'\.LBB\d+_\d+','L',s))
    return out
a=kernels(sys.argv[1]); b=kernels(sys.argv[2])
for k in sorted(set(a)|set(b)):
    if 'rocprim' in k: continue
    if k not in b: print('removed', k[:90]); continue
    if k not in a: print('added', k[:90]); continue
    print('same' if a[k]==b[k] else 'DIFF', len(a[k]), len(b[k]), k[:90])
