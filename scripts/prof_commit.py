#!/usr/bin/env python3
"""Copy one scripts/gpu_profile.sh session directory into the repository (profiles/r0N/prof/prof_NAME) as gzipped
CSVs: bench.json, the kernel-trace CSV and every PMC pass's counter CSV.  --keep-from-dispatch-of K:N keeps, per CSV,
only the rows from the N-th-last group of dispatches of kernel K onwards plus every row of other kernels not named
in --decode (the ~2,000-dispatch IRA decode: the summary reads the last decode only), so the committed copy stays
small; the summary of the copy must equal the summary of the session (checked by the caller).

    python scripts/prof_commit.py gpurun_out/r5prof/prof_c4 profiles/r05/prof/prof_c4 --keep-last k_ira_load:19 \
        --decode k_ira_load,k_ira_vn,k_ira_cn,k_ira_out
"""
import argparse
import csv
import glob
import gzip
import os
import shutil


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--keep-last", help="KERNEL:N — keep the decode rows from the N-th-last dispatch of KERNEL on")
    ap.add_argument("--decode", default="", help="comma list of the decode's kernel name patterns")
    a = ap.parse_args()
    os.makedirs(a.dst, exist_ok=True)
    shutil.copy(os.path.join(a.src, "bench.json"), os.path.join(a.dst, "bench.json"))
    for f in glob.glob(os.path.join(a.src, "**", "*kernel_stats.csv"), recursive=True):  # the rocprofv3 --stats summary
        out = os.path.join(a.dst, os.path.relpath(f, a.src))
        os.makedirs(os.path.dirname(out), exist_ok=True)
        shutil.copy(f, out)
    pats = [p for p in a.decode.split(",") if p]
    files = glob.glob(os.path.join(a.src, "**", "*kernel_trace.csv"), recursive=True)
    files += glob.glob(os.path.join(a.src, "**", "*counter_collection.csv"), recursive=True)
    for f in sorted(files):
        rows = list(csv.DictReader(open(f)))
        if a.keep_last:
            k, n = a.keep_last.rsplit(":", 1)
            ids = sorted({int(r["Dispatch_Id"]) for r in rows if k in r["Kernel_Name"]})
            start = ids[-int(n)] if len(ids) >= int(n) else ids[0]
            rows = [r for r in rows if int(r["Dispatch_Id"]) >= start or not any(p in r["Kernel_Name"] for p in pats)]
        out = os.path.join(a.dst, os.path.relpath(f, a.src) + ".gz")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with gzip.open(out, "wt", newline="") as g:
            w = csv.DictWriter(g, fieldnames=list(rows[0].keys()) if rows else ["Kernel_Name"])
            w.writeheader()
            w.writerows(rows)


if __name__ == "__main__":
    main()
