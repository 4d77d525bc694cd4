#!/usr/bin/env python3
"""Summarise one scripts/gpu_profile.sh session (bench + kernel trace + PMC passes) into a JSON record:
per-launch MEAN counters of the decode and the derived roofline fractions.

    python scripts/counters_summary.py gpurun_out/prof_headline --name headline --kernel k_qc_ms
    python scripts/counters_summary.py gpurun_out/prof_c4 --name c4 --decode-kernels k_load_llr,k_vn_,k_cn_,k_final

Which launches: every profiling pass runs bench.py with ``--steps P --warmup 0`` (P = the number of Eb/N0
points), i.e. the untimed BER pass and the timed loop each launch the decode ONCE PER POINT.  The record
holds the mean over all those launches — each point weighted equally, as in bench's event-timed mean over
a whole number of sweeps — and the kernel-trace pass runs the same arguments, so its mean duration is over
the same launches.  (Round 3 took the median over a 4-step run: for an early-stop kernel that is one
non-converging launch, not the sweep.)  ``--kernel`` names one decode kernel (the register kernels decode
in one launch); ``--decode-kernels`` lists the kernels of a multi-launch decode (generic CSR path): their
counts and durations are summed per decode, decodes = dispatches of the first one.

Derivations (MI355X_MICROARCH.md):
* VALU issue: a wave64 VALU instruction occupies its SIMD-32 for 2 cycles; 1,024 SIMDs.
  valu_frac = 2 * SQ_INSTS_VALU / (1024 * cycles).
* LDS pipe: SQ_LDS_IDX_ACTIVE = LDS-array cycles summed over the 256 CUs. lds_frac = LDS_IDX_ACTIVE / (256 * cycles).
* cycles = GRBM_GUI_ACTIVE / 8: the counter is reported summed over the 8 XCDs (it reads 8 x the launch
  duration x the shader clock).  The clock it implies (cycles / mean kernel-trace duration) must not exceed
  the 2.4 GHz peak engine clock: a record that implies more counted other launches than it timed and is
  REJECTED (exit status 2).
* HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KB; gfx950 FETCH_SIZE counts half the coalesced read bytes;
  re-calibrated in the same pass on k_awgn, whose reads/writes are known exactly).
bench.py reads these per-launch counts and divides them by its live event-timed launch duration.
"""
import argparse
import csv
import glob
import json
import os
import statistics

XCDS, SIMDS, CUS = 8, 1024, 256
MAX_CLOCK_GHZ = 2.4


def per_kernel(path):
    """{(kernel name, counter): [value per dispatch]} over every PMC pass under ``path``."""
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    return vals


def trace_durations(path):
    """{kernel name: [duration ms per dispatch]} from the kernel-trace pass."""
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        for t in csv.DictReader(open(f)):
            out.setdefault(t["Kernel_Name"], []).append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6)
    return out


def summarise(vals, durs, kernel=None, decode_kernels=None):
    """Per-decode counters and duration.  Returns (kernel label, counters, kstats)."""
    if kernel:
        names = {k for (k, _) in vals if kernel in k}
        if not names:
            raise SystemExit(f"no kernel matching {kernel}")
        kname = max(names, key=lambda k: len(vals.get((k, "SQ_INSTS_VALU"), vals.get((k, "FETCH_SIZE"), []))))
        c = {cn: statistics.fmean(v) for (k, cn), v in vals.items() if k == kname}
        d = durs.get(kname, [])
        ks = {"kernel": kname.split("(")[0], "calls": len(d), "mean_ms": statistics.fmean(d) if d else None,
              "min_ms": min(d) if d else None, "max_ms": max(d) if d else None}
        return kname.split("(")[0], c, ks
    pats = decode_kernels.split(",")
    first = [k for k in durs if pats[0] in k]
    if not first:
        raise SystemExit(f"no kernel matching {pats[0]} in the kernel trace")
    n_dec = sum(len(durs[k]) for k in first)
    c = {}
    for (k, cn), v in vals.items():
        if any(p in k for p in pats):
            c[cn] = c.get(cn, 0.0) + sum(v)
    n_dec_pmc = sum(len(v) for (k, cn), v in vals.items() if pats[0] in k and cn in ("FETCH_SIZE", "SQ_INSTS_VALU"))
    n_pmc = {cn: sum(len(v) for (k, c2), v in vals.items() if pats[0] in k and c2 == cn) for cn in c}
    c = {cn: tot / max(n_pmc.get(cn, 0) or n_dec_pmc or 1, 1) for cn, tot in c.items()}
    tot_ms = sum(sum(v) for k, v in durs.items() if any(p in k for p in pats))
    ks = {"kernel": "+".join(pats), "calls": n_dec, "mean_ms": tot_ms / n_dec if n_dec else None,
          "per_kernel_ms": {k.split("(")[0]: statistics.fmean(v) for k, v in durs.items() if any(p in k for p in pats)}}
    return ks["kernel"], c, ks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--name", required=True)
    ap.add_argument("--kernel")
    ap.add_argument("--decode-kernels")
    ap.add_argument("--max-clock-ghz", type=float, default=MAX_CLOCK_GHZ)
    a = ap.parse_args()
    if bool(a.kernel) == bool(a.decode_kernels):
        raise SystemExit("give exactly one of --kernel / --decode-kernels")
    bench = json.load(open(os.path.join(a.dir, "bench.json")))
    vals = per_kernel(a.dir)
    durs = trace_durations(os.path.join(a.dir, "ks"))
    label, c, ks = summarise(vals, durs, a.kernel, a.decode_kernels)
    cfg = bench["config"]
    rec = {"name": a.name, "kernel": label,
           "config": {k: cfg.get(k) for k in ("code", "algo", "iters", "early_stop", "batch_per_gpu", "mod", "kernel_path",
                                              "ebn0", "seed")},
           "launches": "one decode per Eb/N0 point in the BER pass and again in the timed loop (--steps P --warmup 0); "
                       "counters and kernel-trace duration are means over the same launches",
           "bench": {"value": bench["value"], "ms_per_step": bench["ms_per_step"],
                     "launch_ms_events": bench["roofline"]["launch_ms"]},
           "kernel_stats": ks, "counters_per_launch": c}
    d = {}
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / XCDS
        d["cycles"] = cyc
        if ks.get("mean_ms"):
            d["clock_ghz"] = cyc / ks["mean_ms"] / 1e6
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
            d["awgn_fetch_kb_x2"] = 2 * statistics.fmean(vals[(aw[0], "FETCH_SIZE")])
            d["awgn_write_kb"] = statistics.fmean(vals[(aw[0], "WRITE_SIZE")])
    rec["derived"] = d
    if d.get("clock_ghz", 0.0) > a.max_clock_ghz:
        raise SystemExit(f"REJECTED {a.name}: implied clock {d['clock_ghz']:.3f} GHz > {a.max_clock_ghz} GHz — the "
                         f"counted launches are not the timed ones")
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
