"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace (--kernel-trace
--output-format csv).  Prints, per kernel name, the average duration and the average idle time
on the GPU before it starts (time since the previous kernel on the device ended), over the
kernels whose name contains --filter, plus the whole window's busy fraction.

usage: python tools/trace_gaps.py <kernel_trace.csv> [--filter k_] [--last 400]"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("::")[-1][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--filter", default="")
    ap.add_argument("--last", type=int, default=400, help="analyse the last K kernels")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[-a.last:]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    busy = 0
    for s, e, n in rows:
        k = short(n)
        if a.filter in n:
            dur[k].append(e - s)
            if prev_end is not None:
                gap[k].append(max(0, s - prev_end))
        busy += e - s
        prev_end = e if prev_end is None else max(prev_end, e)
    span = rows[-1][1] - rows[0][0]
    print(f"{len(rows)} kernels over {span / 1e3:.1f} us, busy {busy / span:.3f}")
    print(f"{'kernel':62s} {'calls':>5s} {'avg us':>8s} {'gap before us':>13s}")
    for k in dur:
        g = gap[k]
        print(f"{k:62s} {len(dur[k]):5d} {sum(dur[k]) / len(dur[k]) / 1e3:8.1f} "
              f"{(sum(g) / len(g) / 1e3 if g else 0):13.2f}")


if __name__ == "__main__":
    main()
