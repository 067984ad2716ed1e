"""Static views of kernels in a `hipcc --cuda-device-only -S` output (dev tool).

  python tools/isa.py mix    file.s pattern...   instruction mix per kernel
  python tools/isa.py cost   file.s pattern...   static VALU issue cost with the measured gfx950
                                                 rates (tools/microbench/isa_rate.hip: 64-bit ops,
                                                 mads and 32-bit multiplies at half rate; unit =
                                                 one full-rate 32-bit op)
  python tools/isa.py blocks file.s pattern      per-basic-block counts of the first match
  python tools/isa.py res    file.s pattern...   VGPRs, LDS bytes, scratch bytes per kernel (the
                                                 occupancy inputs: 512 / VGPRs waves per SIMD,
                                                 160 KB / LDS workgroups per CU)

A kernel matches when any pattern is a substring of its mangled name."""
import re
import sys
from collections import Counter

HALF = ("v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_lshl_add_u64", "v_cmp_le_u64",
        "v_cmp_lt_u64", "v_cmp_gt_u64", "v_cmp_ge_u64", "v_cmp_gt_i64", "v_cmp_lt_i64",
        "v_lshlrev_b64", "v_lshrrev_b64", "v_mov_b64", "v_cmp_eq_u64", "v_cmp_ne_u64")


def kernels(s, patterns):
    """(mangled name, body lines) of every kernel whose name contains one of `patterns`."""
    for m in re.finditer(r'^(_Z\S+):', s, re.M):
        name = m.group(1)
        if any(p in name for p in patterns):
            body = s[m.end():]
            yield name, body[:body.index('s_endpgm')].split('\n')


def opcodes(lines):
    return [l.strip().split()[0] for l in lines
            if l.startswith('\t') and l.strip() and l.strip()[0] not in ';.']


def mix(s, pats):
    for name, lines in kernels(s, pats):
        c = Counter(opcodes(lines))
        mul = sum(v for k, v in c.items() if 'mul' in k or 'mad' in k)
        print(f"{name[:70]} total={sum(c.values())} "
              f"valu={sum(v for k, v in c.items() if k.startswith('v_'))} mul-class={mul}")
        print('   ' + ', '.join(f'{k}:{v}' for k, v in c.most_common(45)))


def cost(s, pats):
    for name, lines in kernels(s, pats):
        c = Counter(opcodes(lines))
        valu = {k: v for k, v in c.items() if k.startswith('v_')}
        cst = sum(v * (2 if any(k.startswith(h) for h in HALF) else 1) for k, v in valu.items())
        print(f"{name[:60]:60s} VALU={sum(valu.values())} cost={cst} nops={c.get('s_nop', 0)} "
              f"movs={c.get('v_mov_b32_e32', 0)}")


def blocks(s, pats):
    name, lines = next(kernels(s, pats))
    print(name[:100])
    out, cur = [], ['entry', []]
    for l in lines:
        b = re.match(r'^(\.LBB\d+_\d+):', l)
        if b:
            out.append(cur)
            cur = [b.group(1), []]
        else:
            cur[1].extend(opcodes([l]))
    out.append(cur)
    tot = Counter()
    for bname, ins in out:
        c = Counter(ins)
        tot.update(c)
        if ins:
            print(f"{bname:12s} n={len(ins):5d} valu={sum(n for k, n in c.items() if k.startswith('v_')):5d} "
                  f"mad={c['v_mad_u64_u32']:4d} mov={c['v_mov_b32_e32']:4d} nop={c['s_nop']:3d} "
                  f"ds={sum(n for k, n in c.items() if k.startswith('ds_')):3d}")
    print('total', sum(tot.values()), 'valu', sum(n for k, n in tot.items() if k.startswith('v_')))


def res(s, pats):
    # the amdhsa.kernels metadata block: one entry per kernel, fields in alphabetical order
    for m in re.finditer(r'\.group_segment_fixed_size:\s*(\d+).*?\.name:\s*(\S+).*?'
                         r'\.private_segment_fixed_size:\s*(\d+).*?\.vgpr_count:\s*(\d+)', s, re.S):
        lds, name, scratch, vgpr = m.groups()
        if any(p in name for p in pats):
            print(f"{name[:80]:80s} vgpr={vgpr} lds={lds} scratch={scratch}")


if __name__ == "__main__":
    if len(sys.argv) < 4 or sys.argv[1] not in ("mix", "cost", "blocks", "res"):
        sys.exit(__doc__)
    globals()[sys.argv[1]](open(sys.argv[2]).read(), sys.argv[3:])
