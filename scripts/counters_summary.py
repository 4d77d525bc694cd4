#!/usr/bin/env python3
"""Summarise one scripts/gpu_profile.sh session (bench + kernel trace + PMC passes) into a JSON record:
per-launch MEAN counters of the decode and the derived roofline fractions.

    python scripts/counters_summary.py gpurun_out/prof_headline --name headline --kernel k_qc_ms
    python scripts/counters_summary.py gpurun_out/prof_c4 --name c4 --decode-kernels k_load_llr,k_vn_,k_cn_,k_final

Which launches: every profiling pass runs bench.py with ``--steps P --warmup P`` (P = the number of Eb/N0
points): the untimed BER pass, the warmup and the timed loop each launch the decode ONCE PER POINT.  With
``--last P`` the record holds the mean over the timed loop's P launches — each point weighted equally, as in
bench's event-timed mean over a whole number of sweeps, after the clock has ramped — and the kernel-trace
pass runs the same arguments, so its mean duration is over the same launches.  (Round 3 took the median over a 4-step run: for an early-stop kernel that is one
non-converging launch, not the sweep.)  ``--kernel`` names one decode kernel (the register kernels decode
in one launch); ``--decode-kernels`` lists the kernels of a multi-launch decode (generic CSR path): their
counts and durations are summed per decode, decodes = dispatches of the first one.

Derivations (MI355X_MICROARCH.md):
* VALU issue: a wave64 VALU instruction occupies its SIMD-32 for 2 cycles; 1,024 SIMDs.
  valu_frac = 2 * SQ_INSTS_VALU / (1024 * cycles).
* LDS pipe: SQ_LDS_IDX_ACTIVE = LDS-array cycles summed over the 256 CUs. lds_frac = LDS_IDX_ACTIVE / (256 * cycles).
* cycles = GRBM_GUI_ACTIVE / 8: the counter is reported summed over the 8 XCDs (it reads 8 x the launch
  duration x the shader clock).  The clock it implies (cycles / mean kernel-trace duration) must not exceed
  the 2.4 GHz peak engine clock (1 % tolerance: trace timestamps vs the counter's window on the same
  launches): a record that implies more counted other launches than it timed and is REJECTED.
* HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KB; gfx950 FETCH_SIZE counts half the coalesced read bytes;
  re-calibrated in the same pass on k_awgn, whose reads/writes are known exactly).
bench.py reads these per-launch counts and divides them by its live event-timed launch duration.
"""
import argparse
import csv
import glob
import gzip
import json
import os
import statistics

XCDS, SIMDS, CUS = 8, 1024, 256
MAX_CLOCK_GHZ = 2.4
CLOCK_TOL = 1.01  # the trace's timestamps and the counter's GRBM window differ by < 1 % on matching launches


def per_kernel(path):
    """{(kernel name, counter): [[(dispatch id, value)] per PMC pass]} over every pass under ``path`` (each
    pass is its own process, so dispatch ids repeat across passes and are only ordered within one)."""
    vals = {}
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    files += glob.glob(os.path.join(path, "**", "*counter_collection.csv.gz"), recursive=True)  # committed copies
    for f in sorted(files):
        mine = {}
        for r in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
            mine.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append((int(r["Dispatch_Id"]),
                                                                                float(r["Counter_Value"])))
        for k, v in mine.items():
            vals.setdefault(k, []).append(sorted(v))
    return vals


def trace_durations(path, spans=None):
    """{kernel name: [(dispatch id, duration ms)]} from the kernel-trace pass; `spans` (a dict, optional) receives
    {dispatch id: (start ns, end ns)} for the wall span of a multi-launch decode whose dispatches overlap."""
    out = {}
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    files += glob.glob(os.path.join(path, "**", "*kernel_trace.csv.gz"), recursive=True)  # committed copies
    for f in files:
        for t in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
            out.setdefault(t["Kernel_Name"], []).append(
                (int(t["Dispatch_Id"]), (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6))
            if spans is not None:
                spans[int(t["Dispatch_Id"])] = (t["Kernel_Name"], int(t["Start_Timestamp"]), int(t["End_Timestamp"]))
    return {k: sorted(v) for k, v in out.items()}


def _tail(rows, last):
    return [v for _, v in rows[-last:]] if last else [v for _, v in rows]


def summarise(vals, durs, kernel=None, decode_kernels=None, last=0, chunks=1, spans=None):
    """Per-decode counters and duration over the last ``last`` decodes of each pass (0: all), averaged over
    the passes that collected the counter.  ``chunks``: dispatches of the first decode kernel per decode (the
    IRA path launches its load kernel once per Infinity-Cache chunk).  Returns (label, counters, kstats)."""
    if kernel:
        names = {k for (k, _) in vals if kernel in k}
        if not names:
            raise SystemExit(f"no kernel matching {kernel}")
        # the kernel doing the work: most VALU instructions (FETCH_SIZE if no pass counted VALU), not most
        # dispatches — a two-pass decode (the tanh-SP zero pass) dispatches both kernels equally often
        kname = max(sorted(names), key=lambda k: sum(v for pas in vals.get((k, "SQ_INSTS_VALU"), vals.get((k, "FETCH_SIZE"), []))
                                                     for _, v in pas))
        c = {cn: statistics.fmean(statistics.fmean(_tail(rows, last)) for rows in passes)
             for (k, cn), passes in vals.items() if k == kname}
        d = _tail(durs.get(kname, []), last)
        ks = {"kernel": kname.split("(")[0], "calls": len(d), "mean_ms": statistics.fmean(d) if d else None,
              "min_ms": min(d) if d else None, "max_ms": max(d) if d else None}
        return kname.split("(")[0], c, ks
    pats = decode_kernels.split(",")

    def per_decode(rows_by_kernel):
        """(sum over the decode kernels of their values in the last `last` decodes) / decodes, for one pass;
        a decode starts at a dispatch of the first pattern's kernel"""
        ids = sorted(i for k, rows in rows_by_kernel.items() if pats[0] in k for i, _ in rows)
        if not ids:
            raise SystemExit(f"no kernel matching {pats[0]}")
        if len(ids) % chunks:
            raise SystemExit(f"{len(ids)} dispatches of {pats[0]} are not whole decodes of {chunks} chunks")
        ids = ids[::chunks]  # the first chunk's dispatch starts a decode
        start, n_dec = (ids[-last], min(last, len(ids))) if last else (ids[0], len(ids))
        tot = sum(v for k, rows in rows_by_kernel.items() if any(p in k for p in pats) for i, v in rows if i >= start)
        return tot / n_dec, start, n_dec
    c = {}
    for cn in sorted({cn for (_, cn) in vals}):
        npass = max(len(p) for (k, c2), p in vals.items() if c2 == cn)
        per_pass = []
        for ip in range(npass):
            by_k = {k: p[ip] for (k, c2), p in vals.items() if c2 == cn and ip < len(p)}
            per_pass.append(per_decode(by_k)[0])
        c[cn] = statistics.fmean(per_pass)
    tot_ms, start, n_dec = per_decode(durs)
    per = {}
    for k, rows in durs.items():
        if any(p in k for p in pats):
            sel = [v for i, v in rows if i >= start]
            per[k.split("(")[0]] = {"calls": len(sel), "mean_ms": statistics.fmean(sel) if sel else None}
    ks = {"kernel": "+".join(pats), "calls": n_dec, "mean_ms": tot_ms, "per_kernel": per}
    if spans:
        # wall span of each counted decode, first dispatch's start to last dispatch's end: the IRA decode runs its
        # Infinity-Cache chunks on two streams, so its dispatches overlap and the sum of their durations (mean_ms)
        # exceeds the decode's time
        firsts = sorted(i for i, (k, _, _) in spans.items() if pats[0] in k)[::chunks]
        sel = firsts[-n_dec:]
        walls = []
        for j, f in enumerate(sel):
            nxt = sel[j + 1] if j + 1 < len(sel) else None
            ds = [(a, b) for i, (k, a, b) in spans.items() if i >= f and (nxt is None or i < nxt) and any(p in k for p in pats)]
            walls.append((max(b for _, b in ds) - min(a for a, _ in ds)) / 1e6)
        ks["wall_ms"] = statistics.fmean(walls)
    return ks["kernel"], c, ks


def benched_configs():
    """The workloads bench.py reports (the headline, the tanh-SP side number, side.configs' legs): (code, algo, iters,
    early stop, batch per GPU, front end, Eb/N0 grid, seed)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    head = dict(code="wifi648_12", iters=50, early_stop=False, batch=65536, mod="bpsk", ebn0="0:0.5:5")
    out = [dict(head, algo="minsum"), dict(head, algo="tanh")]
    for leg in b.LEGS.values():
        out.append({k: leg[k] for k in ("code", "algo", "iters", "early_stop", "batch", "mod", "ebn0")})
    return out


def benched_mismatch(cfg):
    """None when the profiled run is a configuration bench.py reports, with the library's shipped settings; else why
    not.  The work of a fixed-count decode does not depend on the data, so its record may use fewer Eb/N0 points (the
    PMC passes of config [4]'s five-point grid crashed the profiler, round 5); an early-stop record must have the
    benched grid and seed, since the iterations executed depend on them."""
    if cfg.get("env"):
        return f"run with library overrides {cfg['env']} — not the shipped configuration bench.py times"
    for w in benched_configs():
        if (cfg.get("code"), cfg.get("algo"), cfg.get("iters"), cfg.get("early_stop"), cfg.get("batch_per_gpu"),
                cfg.get("mod")) != (w["code"], w["algo"], w["iters"], w["early_stop"], w["batch"], w["mod"]):
            continue
        if w["early_stop"] and (cfg.get("ebn0") != w["ebn0"] or cfg.get("seed") != 2024):
            return f"early stop with Eb/N0 {cfg.get('ebn0')} / seed {cfg.get('seed')}: the benched run uses {w['ebn0']} / 2024"
        return None
    return f"{cfg.get('code')} {cfg.get('algo')} {cfg.get('iters')} it, B {cfg.get('batch_per_gpu')}: not a configuration bench.py reports"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--name", required=True)
    ap.add_argument("--kernel")
    ap.add_argument("--chunks", type=int, default=1, help="first-decode-kernel dispatches per decode")
    ap.add_argument("--decode-kernels")
    ap.add_argument("--max-clock-ghz", type=float, default=MAX_CLOCK_GHZ)
    ap.add_argument("--last", type=int, default=0, help="use the last N decodes of each pass (the timed loop)")
    a = ap.parse_args()
    if bool(a.kernel) == bool(a.decode_kernels):
        raise SystemExit("give exactly one of --kernel / --decode-kernels")
    bench = json.load(open(os.path.join(a.dir, "bench.json")))
    why = benched_mismatch(bench["config"])
    if why:
        raise SystemExit(f"REJECTED {a.name}: {why}")
    vals = per_kernel(a.dir)
    spans = {} if a.decode_kernels else None
    durs = trace_durations(os.path.join(a.dir, "ks"), spans)
    label, c, ks = summarise(vals, durs, a.kernel, a.decode_kernels, a.last, a.chunks, spans)
    cfg = bench["config"]
    rec = {"name": a.name, "kernel": label,
           "config": {k: cfg.get(k) for k in ("code", "algo", "iters", "early_stop", "batch_per_gpu", "mod", "kernel_path",
                                              "ebn0", "seed", "env")},
           "clock": bench.get("clock"),
           "launches": f"the timed loop of `--steps P --warmup P` (P = Eb/N0 points): the last {a.last} decodes, one per "
                       "point; counters and kernel-trace duration are means over the same launches",
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
            d["awgn_fetch_kb_x2"] = 2 * statistics.fmean(_tail(vals[(aw[0], "FETCH_SIZE")][0], 0))
            d["awgn_write_kb"] = statistics.fmean(_tail(vals[(aw[0], "WRITE_SIZE")][0], 0))
    rec["derived"] = d
    # a multi-launch decode adds each dispatch's few us of front-end time to the counter's window but not to the
    # kernels' traced durations: 3 % at ~500 dispatches (the generic kernels), more for the IRA decode's ~1,900;
    # allowed: 8 us per dispatch on top of 3 % (counting the wrong launches would still be 2x off)
    if a.kernel:
        tol = CLOCK_TOL
    else:
        per_dec = sum(v["calls"] for v in ks["per_kernel"].values()) / max(1, ks["calls"])
        tol = 1.03 + (per_dec * 8e-3 / ks["mean_ms"] if ks.get("mean_ms") else 0.0)
        d["dispatches_per_decode"] = per_dec
    if d.get("clock_ghz", 0.0) > a.max_clock_ghz * tol:
        raise SystemExit(f"REJECTED {a.name}: implied clock {d['clock_ghz']:.3f} GHz > {a.max_clock_ghz} GHz — the "
                         f"counted launches are not the timed ones")
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
