"""Per-basic-block instruction counts of one kernel in a hipcc -S output (dev tool).
usage: python tools/isa_blocks.py file.s symbol-substring"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
m = re.search(r'^(_Z\S*' + re.escape(sys.argv[2]) + r'\S*):', s, re.M)
body = s[m.end():]
body = body[:body.index('s_endpgm')]
blocks, cur = [], ['entry', []]
for l in body.split('\n'):
    b = re.match(r'^(\.LBB\d+_\d+):', l)
    if b:
        blocks.append(cur)
        cur = [b.group(1), []]
    elif l.startswith('\t') and l.strip() and l.strip()[0] not in ';.':
        cur[1].append(l.strip().split()[0])
blocks.append(cur)
tot = Counter()
for name, ins in blocks:
    c = Counter(ins)
    tot.update(c)
    v = sum(n for k, n in c.items() if k.startswith('v_'))
    if not ins:
        continue
    print(f"{name:12s} n={len(ins):5d} valu={v:5d} mad={c['v_mad_u64_u32']:4d} "
          f"mov={c['v_mov_b32_e32']:4d} nop={c['s_nop']:3d} ds={sum(n for k, n in c.items() if k.startswith('ds_')):3d}")
print('total', sum(tot.values()), 'valu', sum(n for k, n in tot.items() if k.startswith('v_')))
