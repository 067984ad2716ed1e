"""Static VALU cost of kernels in a hipcc -S output using the measured gfx950 issue costs
(tools/microbench/isa_rate.hip; unit = one full-rate 32-bit VALU op).  Dev tool.
usage: python tools/isa_cost.py file.s pattern..."""
import re, sys
from collections import Counter
HALF = ("v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_lshl_add_u64", "v_cmp_le_u64", "v_cmp_lt_u64",
        "v_cmp_gt_u64", "v_cmp_ge_u64", "v_cmp_gt_i64", "v_cmp_lt_i64", "v_lshlrev_b64", "v_lshrrev_b64",
        "v_mov_b64", "v_cmp_eq_u64", "v_cmp_ne_u64")
s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_Z\S+):', s, re.M):
    name = m.group(1)
    if not any(p in name for p in sys.argv[2:]):
        continue
    body = s[m.end():]
    body = body[:body.index('s_endpgm')]
    ins = [l.split()[0] for l in body.split('\n') if l.startswith('\t') and l.strip() and l.strip()[0] not in ';.']
    c = Counter(ins)
    valu = {k: v for k, v in c.items() if k.startswith('v_')}
    cost = sum(v * (2 if any(k.startswith(h) for h in HALF) else 1) for k, v in valu.items())
    print(f"{name[:60]:60s} VALU={sum(valu.values())} cost={cost} nops={c.get('s_nop',0)} movs={c.get('v_mov_b32_e32',0)}")
