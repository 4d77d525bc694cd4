#!/usr/bin/env python3
"""Per-kernel summary of scripts/kprof.sh: dispatches, mean duration (kernel trace) and the mean of every collected
counter per dispatch, with HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KB; gfx950 FETCH_SIZE halves coalesced reads)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "ks", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            cnt[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    tot = sum(sum(v) for v in dur.values())
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        v = dur[k]
        line = f"{k[:70]:70s} n={len(v):5d} mean={sum(v)/len(v):9.4f} ms total={sum(v):8.2f} ms ({100*sum(v)/tot:5.1f}%)"
        c = {n: sum(x) / len(x) for n, x in cnt.get(k, {}).items()}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hb = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            line += f" hbm={hb/1e6:8.2f} MB ({hb / (sum(v)/len(v)*1e-3) / 1e12:5.2f} TB/s)"
        for n in sorted(c):
            line += f" {n}={c[n]:.4g}"
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
            line += f" l2hit={c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
