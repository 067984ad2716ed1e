"""Compare tools/pmc_stall.sh outputs of several builds per kernel: time, effective clock (GRBM
cycles per XCD / time), VALU instructions per wave, wave-state split.  Dev tool.
usage: python tools/pmc_compare.py <outdir> tag [tag ...]"""
import csv, glob, os, sys
from collections import defaultdict

def short(n):
    n = n.replace("void fhe::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]

def load(d):
    st, vals = {}, defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            st[short(r["Name"])] = float(r["AverageNs"])
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return st, {k: {c: sum(v) / len(v) for c, v in d2.items()} for k, d2 in vals.items()}

out, tags = sys.argv[1], sys.argv[2:]
data = {t: load(os.path.join(out, t)) for t in tags}
kernels = sorted(set().union(*[set(d[0]) for d in data.values()]))
print(f"{'kernel':28s} {'build':8s} {'us':>7s} {'GHz':>5s} {'valu/wave':>9s} {'active':>6s} {'waitinst':>8s} {'waitany':>7s} {'waves/SIMD':>10s}")
for k in kernels:
    if not k.startswith("k_"):
        continue
    for t in tags:
        st, v = data[t]
        if k not in st or k not in v:
            continue
        c = v[k]
        us = st[k] / 1e3
        ghz = c.get("GRBM_GUI_ACTIVE", 0) / 8 / (us * 1e3)
        w = c.get("SQ_WAVE_CYCLES", 1)
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        print(f"{k[:28]:28s} {t[:8]:8s} {us:7.1f} {ghz:5.2f} {c.get('SQ_INSTS_VALU',0)/c.get('SQ_WAVES',1):9.0f} "
              f"{c.get('SQ_ACTIVE_INST_ANY',0)/w:6.2f} {c.get('SQ_WAIT_INST_ANY',0)/w:8.2f} {c.get('SQ_WAIT_ANY',0)/w:7.2f} "
              f"{4*w/1024/cyc if cyc else 0:10.2f}")
