#!/usr/bin/env python3
"""Mean duration of the decode kernel's TIMED launches in a rocprofv3 --kernel-trace run of bench.py: the
last `steps` dispatches of the kernel (bench.py launches the untimed BER sweep and the warmup first), next
to the --stats average over every dispatch.  Reconciles the profiler with bench's event-timed launch_ms.

    python scripts/timed_launches.py <session dir with ks/*kernel_trace.csv and bench.json> --kernel k_qc_ms_ph
"""
import argparse
import csv
import glob
import json
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("session")
ap.add_argument("--kernel", required=True)
a = ap.parse_args()
bench = json.load(open(os.path.join(a.session, "bench.json")))
steps = int(bench["steps"])
rows = []
for f in glob.glob(os.path.join(a.session, "**", "*kernel_trace.csv"), recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if a.kernel in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
timed = d[-steps:]
print(json.dumps({"session": os.path.basename(os.path.normpath(a.session)), "kernel": a.kernel, "dispatches": len(d),
                  "all_mean_ms": statistics.fmean(d), "timed_steps": steps, "timed_mean_ms": statistics.fmean(timed),
                  "timed_min_ms": min(timed), "timed_max_ms": max(timed),
                  "bench_launch_ms": bench["roofline"]["launch_ms"], "bench_ms_per_step": bench["ms_per_step"]}))
