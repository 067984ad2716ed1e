"""Instruction mix of kernels in a hipcc -S output (dev tool).
usage: python tools/isa_mix.py file.s pattern [pattern...]"""
import re, sys
from collections import Counter
s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_Z\S+):', s, re.M):
    name = m.group(1)
    if not any(p in name for p in sys.argv[2:]):
        continue
    body = s[m.end():]
    body = body[:body.index('s_endpgm')]
    ins = [l.split()[0] for l in body.split('\n') if l.startswith('\t') and l.strip() and not l.strip()[0] in ';.']
    c = Counter(ins)
    mul = sum(v for k, v in c.items() if 'mul' in k or 'mad' in k)
    print(f"{name[:70]} total={len(ins)} mul-class={mul}")
    print('   ' + ', '.join(f'{k}:{v}' for k, v in c.most_common(45)))
    meta = re.search(re.escape(name) + r'.*?\.vgpr_count:\s+(\d+)', s[m.end():], re.S)
