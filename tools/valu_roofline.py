"""Counter-based VALU roofline per kernel from a tools/pmc_stall.sh bundle (dev / measurement tool).

For every kernel of the profiled command: launches, mean duration (the --kernel-trace pass),
SQ_INSTS_VALU per launch (wave-level VALU instructions, the pmc1 pass), effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration) and the achieved VALU issue rate.  The ceiling is the issue
rate of tools/microbench/bfly_peak.hip (the row passes' butterfly sequences, register-resident, no
memory traffic) measured in the same profiled process, so frac = achieved / that rate: how close a
kernel's instruction stream runs to what the chip sustains on pure 64-bit modular arithmetic.

usage: python tools/valu_roofline.py <bundle>/<tag> [out.json] [--steps S] [--batch B]
  --steps S: steps the profiled command ran (warmup + timed): launches_per_step = launches / S;
  --batch B: the per-call batch of the profiled shape (recorded for bench.py's shape match)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void fhe::(anonymous namespace)::", "").replace("void (anonymous namespace)::", "")
    return n.split("(")[0]


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    opt = {a: int(b) for a, b in zip(sys.argv, sys.argv[1:]) if a in ("--steps", "--batch")}
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc1", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            cnt[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, c in cnt.items():
        if k not in dur or "SQ_INSTS_VALU" not in c:
            continue
        us = sum(dur[k]) / len(dur[k])
        valu = sum(c["SQ_INSTS_VALU"]) / len(c["SQ_INSTS_VALU"])
        waves = sum(c["SQ_WAVES"]) / len(c["SQ_WAVES"]) if "SQ_WAVES" in c else None
        grbm = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"]) if "GRBM_GUI_ACTIVE" in c else 0
        res[k] = {"launches": len(dur[k]), "mean_us": round(us, 2),
                  "valu_instr_per_launch": valu,
                  "valu_per_wave": round(valu / waves, 1) if waves else None,
                  # GRBM_GUI_ACTIVE over a launch shorter than ~10 us counts mostly the
                  # dispatch and drain around it: no meaningful clock (r5 verdict: 8-14 "GHz")
                  "clock_ghz": round(grbm / 8 / (us * 1e3), 3) if grbm and us >= 10 else None,
                  "valu_g_per_s": round(valu / (us * 1e3), 2)}
    peak = [v["valu_g_per_s"] for k, v in res.items() if k.startswith("k_bfly_peak")]
    ceiling = max(peak) if peak else None
    for k, v in res.items():
        if ceiling and k.startswith("k_"):
            v["frac_of_bfly_peak_issue"] = round(v["valu_g_per_s"] / ceiling, 4)
        if "--steps" in opt:
            v["launches_per_step"] = v["launches"] / opt["--steps"]
    rec = {"source": d, "shape": {"batch": opt.get("--batch")}, "ceiling_valu_g_per_s": ceiling,
           "ceiling_kernel": "k_bfly_peak (tools/microbench/bfly_peak.hip), same profiled process",
           "kernels": res}
    js = json.dumps(rec, indent=1)
    if out:
        open(out, "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
