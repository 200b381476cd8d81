# Dev tool: per-kernel instruction mix of a device .s file (hipcc --cuda-device-only -S).
# usage: python profiles/tools_isa.py <file.s> <kernel-name regex> [count]
import re, sys
from collections import Counter
s = open(sys.argv[1]).read()
pat = sys.argv[2]
names = [m for m in re.findall(r'^(_Z\S*):\n', s, re.M) if re.search(pat, m)]
for name in names[:int(sys.argv[3]) if len(sys.argv) > 3 else 1]:
    start = s.index(name + ':\n')
    end = s.index('.Lfunc_end', start)
    body = s[start:end].splitlines()
    ins = [l.strip() for l in body if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
    c = Counter()
    for i in ins:
        op = i.split()[0]
        cat = 'valu' if op.startswith('v_') else 'salu' if op.startswith('s_') else 'lds' if op.startswith('ds_') else 'vmem' if op.startswith(('global_', 'buffer_', 'flat_', 'scratch_')) else 'other'
        c[cat] += 1
    print(name[:90], len(ins), dict(c))
    print(Counter(i.split()[0] for i in ins).most_common(40))
