#!/usr/bin/env python3
"""Summarise one scripts/gpu_profile.sh session (bench + kernel stats + PMC passes) into a JSON record:
per-launch means of the decode kernel's counters and the derived roofline fractions.

    python scripts/counters_summary.py gpurun_out/prof_headline --name headline --kernel k_qc_ms

Derivations (MI355X_MICROARCH.md):
* VALU issue: a wave64 VALU instruction occupies its SIMD-32 for 2 cycles; 1,024 SIMDs.
  valu_frac = 2 * SQ_INSTS_VALU / (1024 * cycles).
* LDS pipe: SQ_LDS_IDX_ACTIVE = LDS-array cycles summed over the 256 CUs. lds_frac = LDS_IDX_ACTIVE / (256 * cycles).
* cycles = GRBM_GUI_ACTIVE / 8: the counter is reported summed over the 8 XCDs (it reads 8 x the launch
  duration x the shader clock).  The clock it implies is recorded as clock_ghz.
* HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KB; gfx950 FETCH_SIZE counts half the coalesced read bytes;
  re-calibrated in the same pass on k_awgn, whose reads/writes are known exactly).
bench.py reads these per-launch instruction / cycle counts (deterministic for a fixed iteration count)
and divides them by its live event-timed launch duration.
"""
import argparse
import csv
import glob
import json
import os
import statistics

XCDS, SIMDS, CUS = 8, 1024, 256


def per_kernel(path):
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    return vals


def kstats(path, key):
    f = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
    rows = [r for r in csv.DictReader(open(f[0]))] if f else []
    rows = [r for r in rows if key in r["Name"]]
    if not rows:
        return None
    r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    trace = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    durs = []
    if trace:
        for t in csv.DictReader(open(trace[0])):
            if t["Kernel_Name"] == r["Name"]:
                durs.append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6)
    return {"kernel": r["Name"].split("(")[0], "calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
            "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6,
            "median_ms": statistics.median(durs) if durs else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--name", required=True)
    ap.add_argument("--kernel", required=True)
    a = ap.parse_args()
    bench = json.load(open(os.path.join(a.dir, "bench.json")))
    ks = kstats(os.path.join(a.dir, "ks"), a.kernel)
    vals = per_kernel(a.dir)
    kern = [k for (k, c) in vals if a.kernel in k]
    if not kern:
        raise SystemExit(f"no kernel matching {a.kernel}")
    kname = max(set(kern), key=lambda k: len(vals.get((k, "SQ_INSTS_VALU"), [])))
    c = {cn: statistics.median(v) for (k, cn), v in vals.items() if k == kname}
    cfg = bench["config"]
    rec = {"name": a.name, "kernel": kname.split("(")[0],
           "config": {k: cfg.get(k) for k in ("code", "algo", "iters", "early_stop", "batch_per_gpu", "mod", "kernel_path",
                                                      "ebn0", "seed")},
           "bench": {"value": bench["value"], "ms_per_step": bench["ms_per_step"],
                     "launch_ms_events": bench["roofline"]["launch_ms"]},
           "kernel_stats": ks, "counters_per_launch": c}
    d = {}
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / XCDS
        d["cycles"] = cyc
        if ks:
            d["clock_ghz"] = cyc / (ks["median_ms"] or ks["avg_ms"]) / 1e6
        if "SQ_INSTS_VALU" in c:
            d["valu_frac"] = 2 * c["SQ_INSTS_VALU"] / (SIMDS * cyc)
        if "SQ_LDS_IDX_ACTIVE" in c:
            d["lds_frac"] = c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c and "SQ_WAVE_CYCLES" in c:
                d[k.lower() + "_over_wave_cycles"] = c[k] / c["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
        d["valu_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        d["lds_per_wave"] = c.get("SQ_INSTS_LDS", 0) / c["SQ_WAVES"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        d["hbm_bytes"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        aw = [k for (k, cn) in vals if "k_awgn" in k and cn == "FETCH_SIZE"]
        if aw:
            d["awgn_fetch_kb_x2"] = 2 * statistics.median(vals[(aw[0], "FETCH_SIZE")])
            d["awgn_write_kb"] = statistics.median(vals[(aw[0], "WRITE_SIZE")])
    rec["derived"] = d
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
