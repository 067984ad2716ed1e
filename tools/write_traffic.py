"""Turn a tools/profile_round.sh bundle into profiles/: the rocprofv3 kernel stats, the PMC traffic
summary and profiles/hbm_traffic.json (bytes per launch of bench.py's dominant kernel, read from the
memory-side counters and corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE counts half
the bytes of these streaming reads on gfx950 -- verified here against the column pass, whose
algorithmic traffic is known, in tools/pmc_traffic.sh -- WRITE_SIZE counts them exactly).
usage: python tools/write_traffic.py <bundle dir> <round tag>"""
import csv, glob, json, os, shutil, sys
from collections import defaultdict

bundle, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")


def short(n):
    return n.replace("void fhe::(anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0]


vals = defaultdict(lambda: defaultdict(list))
for part in ("fetch", "write"):
    for f in glob.glob(os.path.join(bundle, part, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[(short(r["Kernel_Name"]), int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
bench = json.load(open(os.path.join(bundle, "bench.json")))
rows = []
for (k, g), d in sorted(vals.items()):
    if "k_" not in k:
        continue
    rd = 2 * 1024 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
    wr = 1024 * sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
    rows.append({"kernel": k, "grid": g, "read_bytes": int(rd), "write_bytes": int(wr),
                 "launches": len(d["FETCH_SIZE"])})
cfg = bench["config"]
shape = {"log_n": cfg["log_n"], "batch": cfg["global_batch"], "nlimbs": cfg["limbs"] // bench["n_gpus"]}
hm = [r for r in rows if r["kernel"].startswith("k_hommult_row")]
out = {"_source": f"profiles/{tag}_pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of "
                  f"`python bench.py`); read = 2 x FETCH_SIZE, write = WRITE_SIZE",
       "hm_row_tensor": {"shape": shape, "bytes_per_launch": hm[0]["read_bytes"] + hm[0]["write_bytes"],
                         "read_bytes": hm[0]["read_bytes"], "write_bytes": hm[0]["write_bytes"]}}
json.dump(out, open(os.path.join(prof, "hbm_traffic.json"), "w"), indent=1)
json.dump(rows, open(os.path.join(prof, f"{tag}_pmc_traffic.json"), "w"), indent=1)
shutil.copy(os.path.join(bundle, "stats", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
shutil.copy(os.path.join(bundle, "bench.json"), os.path.join(prof, f"{tag}_bench.json"))
print(json.dumps(out, indent=1))
