"""Summarise rocprofv3 kernel-trace stats + PMC passes written by tools/pmc.sh (dev tool).
usage: python tools/pmc_summary.py <outdir> [kernel-substring ...]"""
import csv, glob, os, sys
from collections import defaultdict
out = sys.argv[1]
pats = sys.argv[2:] or ["k_"]
def short(n):
    n = n.replace("void fhe::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]
stats = {}
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        stats[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(set(stats) | set(vals)):
    if not any(p in k for p in pats):
        continue
    calls, avg = stats.get(k, (0, float("nan")))
    print(f"== {k}  calls={calls} avg={avg/1e3:.2f} us")
    row = {c: sum(v) / len(v) for c, v in vals[k].items()}
    for c in sorted(row):
        print(f"   {c:28s} {row[c]:.4g}")
