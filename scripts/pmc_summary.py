#!/usr/bin/env python3
"""Summarise the PMC HBM-traffic passes of scripts/gpu_pmc.sh into profiles/pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE are in KB per dispatch, summed over the TCC channels.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half of the coalesced read bytes -> x2; WRITE_SIZE
is exact.  The correction is re-checked in the same run on k_awgn, whose traffic is known exactly
(reads B*n codeword bytes, writes B*n float32 LLRs).

    python scripts/pmc_summary.py gpurun_out [--code wifi648_12 --batch 65536 --iters 50]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_kernel(path):
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def pick(vals, key):
    ks = [k for k in vals if key in k]
    if not ks:
        raise SystemExit(f"no kernel matching {key}")
    k = max(ks, key=lambda k: len(vals[k]))
    return k, statistics.median(vals[k])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--code", default="wifi648_12")
    ap.add_argument("--n", type=int, default=648)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--kernel", default="k_qc_ms")
    ap.add_argument("--dest", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                                                    "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = per_kernel(os.path.join(a.out, "pmc_FETCH_SIZE"))
    write = per_kernel(os.path.join(a.out, "pmc_WRITE_SIZE"))
    kname, f_kb = pick(fetch, a.kernel)
    _, w_kb = pick(write, a.kernel)
    _, fa = pick(fetch, "k_awgn")
    _, wa = pick(write, "k_awgn")
    B, n = a.batch, a.n
    awgn_read, awgn_write = B * n, B * n * 4
    hbm = 2 * f_kb * 1024 + w_kb * 1024
    rec = dict(code=a.code, batch=B, iters=a.iters, algo="minsum", path="qc", kernel=kname.split("(")[0],
               fetch_size_kb_raw=f_kb, write_size_kb_raw=w_kb,
               correction=(f"MI355X_MICROARCH.md HBM: FETCH_SIZE reads 1/2 of coalesced read bytes on gfx950 -> x2; "
                           f"WRITE_SIZE exact. Calibrated in the same run on k_awgn: reads {awgn_read:,} B of codewords "
                           f"-> FETCH {fa:.0f} KB (x2 = {2 * fa:.0f} KB vs {awgn_read / 1024:.0f} KB), writes "
                           f"{awgn_write:,} B -> WRITE {wa:.0f} KB ({awgn_write / 1024:.0f} KB)."),
               hbm_bytes_per_launch=hbm, algorithmic_io_bytes=B * n * 4 + B * n,
               source=f"{a.out}/pmc_*/ (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py)")
    with open(a.dest, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
