"""Instruction mix of the innermost MFMA loop of a kernel in a hipcc -S listing: isa_loop.py <file.s> <symbol>."""
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
a = s.index(name + ':')
b = s.index('.Lfunc_end', a)
body = s[a:b].split('\n')
mf = [i for i, l in enumerate(body) if 'v_mfma' in l]
labels = [i for i, l in enumerate(body) if l.strip().startswith('.LBB') and l.strip().endswith(':')]
lo = [i for i in labels if i < mf[0]][-1]
hi = [i for i, l in enumerate(body) if i > mf[-1] and ('s_cbranch' in l or 's_branch' in l)][0]
cnt = {}
for l in body[lo:hi + 1]:
    t = l.strip().split()
    if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
        continue
    cnt[t[0]] = cnt.get(t[0], 0) + 1
print('loop lines %d-%d: %d instructions, %d mfma' % (lo, hi, sum(cnt.values()), cnt.get(next((k for k in cnt if 'mfma' in k), ''), 0)))
for k, v in sorted(cnt.items(), key=lambda x: -x[1]):
    print('%5d %s' % (v, k))
