#!/usr/bin/env python3
"""Headline benchmark: decoded codewords/s + BER vs Eb/N0, 802.11n (648,1/2), min-sum, 50 iterations.

One step = one decode of a batch of B = 65,536 codewords (per GPU) of one Eb/N0 point, LLRs already
resident in HBM; steps cycle through the 11 points Eb/N0 = 0:0.5:5 dB (BASELINE.json configs[1]).
Before timing, one untimed pass over all 11 points produces the BER/BLER curve (error counts on device,
summed over ranks with an RCCL all-reduce — the only collective; the codeword batches shard with no
data-path exchange, so scaling is weak).

    python bench.py [--gpus N --steps K --warmup W]                  # N=1
    torchrun --nproc-per-node N ... bench.py --gpus N ...            # one rank per GPU

The other BASELINE.json configs are parity-test cases; their throughput lines (profiles/) come from
the same script, e.g. configs[2]: --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9;
configs[3]: --code wifi1296_23 --algo qminsum --iters 20 --early-stop; configs[4]: --code dvbs2_12 --batch 4096 (EN 302 307 rate-1/2 table).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ldpc-sims_amd"))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes_per_cw(n, E, iters, s_m=4, s_l=4):
    """the reference's two-array flooding dataflow per codeword:
    iters*(4*E*s_m + n*s_L) + n*s_L + n."""
    return iters * (4 * E * s_m + n * s_l) + n * s_l + n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=22)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--code", default="wifi648_12")
    ap.add_argument("--algo", default="minsum")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=65536, help="codewords per GPU per step")
    ap.add_argument("--clamp", type=float, default=20.0)
    ap.add_argument("--alpha", type=float, default=1.0)
    ap.add_argument("--ebn0", default="0:0.5:5")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--force-generic", action="store_true")
    ap.add_argument("--early-stop", action="store_true", help="syndrome early termination (cw/s then depends on Eb/N0)")
    ap.add_argument("--qstep", type=float, default=1.0, help="qminsum: LLR quantisation step (5-bit: qmax 15)")
    ap.add_argument("--mod", default="bpsk", choices=["bpsk", "qpsk-ofdm", "16qam-ofdm"],
                    help="LLR generator (outside the timed region): BPSK/AWGN or the OFDM front end")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the decode_bits / tanh-SP side measurements")
    ap.add_argument("--ref-cpu-json", default=os.path.join(ROOT, "profiles", "ref_cpu_wifi648.json"),
                    help="the reference's own CPU decode_bits timing (scripts/time_reference_cpu.py)")
    ap.add_argument("--counters-json", default=os.path.join(ROOT, "profiles", "counters.json"),
                    help="per-launch PMC counts per configuration (scripts/gpu_profile.sh + counters_summary.py)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import ldpc_amd
    from ldpc_amd import _abi
    from ldpc_amd.dist import allreduce_counts, max_over_ranks
    from ldpc_amd.synth import DeviceEncoder

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LDPC_BENCH_BACKEND / device modulo exist only to rehearse N>1 on a 1-GPU box (ranks share cuda:0,
    # counters over gloo); the driver's multi-GPU runs use the defaults: one GPU per rank, RCCL.
    local = local % max(1, torch.cuda.device_count()) if os.environ.get("LDPC_BENCH_SHARE_GPU") else local
    torch.cuda.set_device(local)
    if world > 1:
        backend = os.environ.get("LDPC_BENCH_BACKEND", "nccl")  # nccl == RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    H, qc = ldpc_amd.get_code(args.code)
    m, n = H.shape
    k = n - m
    rate = k / n
    dec = ldpc_amd.get_decoder(H, local)
    B = args.batch
    lo, step_db, hi = (float(x) for x in args.ebn0.split(":"))
    ebn0 = np.round(np.arange(lo, hi + 1e-9, step_db), 6)
    lib = _abi.load()
    stream = torch.cuda.current_stream()
    st = stream.cuda_stream

    # ---- synthetic data, resident in HBM before timing -------------------------------------------
    enc = DeviceEncoder(H, torch.device("cuda", local))
    info = torch.empty((B, k), dtype=torch.uint8, device="cuda")
    _abi.check(lib.ldpc_random_bits(info.data_ptr(), B, k, args.seed, rank * B, st))
    cw = enc.encode(info)
    llrs = []
    for i, e in enumerate(ebn0):
        x = torch.empty((B, n), dtype=torch.float32, device="cuda")
        if args.mod == "bpsk":
            sigma = float(np.sqrt(1.0 / (2.0 * rate * 10.0 ** (e / 10.0))))
            _abi.check(lib.ldpc_awgn_llr(cw.data_ptr(), x.data_ptr(), B, n, sigma, args.seed * 1000 + i, rank * B, st))
        else:
            from ldpc_amd.channel import ofdm_demod, ofdm_tx
            bps = 2 if args.mod == "qpsk-ofdm" else 4
            esn0 = float(10.0 ** (e / 10.0) * rate * bps)
            s_ = cw.view(-1)
            pad = (-s_.numel()) % (bps * 32)
            if pad:
                s_ = torch.cat([s_, torch.zeros(pad, dtype=torch.uint8, device="cuda")])
            rx = ofdm_tx(s_, 32, bps, esn0, args.seed * 1000 + i, rank * B * n // bps)
            x.copy_(ofdm_demod(rx, 32, bps, esn0)[:B * n].view(B, n))
        llrs.append(x)
    p = dec.params(args.iters, args.algo, args.clamp, args.alpha, 0.0, args.early_stop, "f32", "p1",
                   qstep=args.qstep, force_generic=args.force_generic, device_ptrs=True)
    wsb = dec.workspace_bytes(B, p)
    ws = torch.empty((wsb,), dtype=torch.uint8, device="cuda")
    bits = torch.empty((B, n), dtype=torch.uint8, device="cuda")

    def step(x):
        _abi.check(lib.ldpc_decode_ex(dec._h, x.data_ptr(), B, p, bits.data_ptr(), None, None, ws.data_ptr(), wsb, st))

    # ---- BER sweep (untimed; also warms up) --------------------------------------------------------
    counts = torch.zeros((len(ebn0), 3), dtype=torch.int64, device="cuda")
    for i in range(len(ebn0)):
        step(llrs[i])
        _abi.check(lib.ldpc_count_errors(bits.data_ptr(), cw.data_ptr(), B, n, k, counts[i].data_ptr(), st))
    allreduce_counts(counts)  # the one collective: per-point error counters, 24 B x 11 per rank (RCCL)
    c = counts.cpu().numpy().astype(np.float64)
    coded_ber = (c[:, 0] / (c[:, 2] * k)).tolist()
    coded_bler = (c[:, 1] / c[:, 2]).tolist()
    for w in range(args.warmup):
        step(llrs[w % len(ebn0)])
    torch.cuda.synchronize()

    # ---- timed region -------------------------------------------------------------------------------
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for s in range(args.steps):
        step(llrs[s % len(ebn0)])
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    gpu_ms = ev0.elapsed_time(ev1) / max(args.steps, 1)
    my_elapsed = elapsed
    elapsed = max_over_ranks(elapsed, device="cuda")
    total_cw = world * args.steps * B
    ranks = rank_evidence(world, rank, local, my_elapsed)
    value = total_cw / elapsed

    # ---- roofline ---------------------------------------------------------------------------------------
    E = int(H.sum())  # nnz (SparseCode.sum() too)
    kpath = "generic-csr" if (args.force_generic or not dec.qc_z) else f"qc-z{dec.qc_z}"
    roof = roofline(n, E, B, gpu_ms, args, kpath)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # CPU baseline at N=1 only
        cpu = cpu_baseline(H, args, rate)
    side = None
    if rank == 0 and world == 1 and not args.no_dropin and B * n * 8 <= (1 << 32):
        side = side_measurements(H, dec, llrs[len(ebn0) // 2], B, args)
        ref = reference_cpu(args)
        if cpu is not None and ref is not None:
            if "value" in ref:
                ref["gpu_tanh_sp_over_reference"] = side["gpu_tanh_sp"]["cw_per_s"] / ref["value"]
                ref["dropin_over_reference"] = side["dropin"]["cw_per_s"] / ref["value"]
                ref["headline_over_reference"] = value / ref["value"]
            cpu["reference"] = ref

    if rank == 0:
        out = {
            "metric": "decoded codewords/sec + BER@Eb/N0 sweep, (648,1/2) 50-iter min-sum",
            "value": value,
            "unit": "codewords/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: random info bits, systematic encoder, {args.mod} LLRs generated on device",
            "config": {
                "workload": f"{args.code} {args.algo} {args.iters} iters{' early-stop' if args.early_stop else ''}, "
                            f"B={B} codewords/GPU/step, Eb/N0 {args.ebn0} dB cycled per step",
                "code": args.code, "n": n, "k": k, "edges": E, "algo": args.algo, "iters": args.iters,
                "clamp": args.clamp, "alpha": args.alpha, "early_stop": args.early_stop, "mod": args.mod,
                "ebn0": args.ebn0, "seed": args.seed,
                "batch_per_gpu": B, "global_batch": B * world,
                "parallelism": f"dp{world} (codeword shards, RCCL all-reduce of error counts only)",
                "kernel_path": kpath,
            },
            "ranks": ranks,
            "roofline": roof,
            "cpu_baseline": cpu,
            "dropin_cw_per_s": side["dropin"]["cw_per_s"] if side else None,
            "side": side,
            "ber": {"ebn0_db": ebn0.tolist(), "coded_ber_info": coded_ber, "coded_bler": coded_bler,
                    "codewords_per_point": int(c[0, 2])},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rank_evidence(world, rank, local, elapsed):
    """What the process group itself reports: world size and backend from torch.distributed, and every
    rank's device (index, name, PCI bus, UUID) and timed-region seconds, gathered to rank 0 over the same
    group (the counter all-reduce's), so a multi-GPU record shows that RCCL saw N ranks on N GPUs."""
    import torch
    import torch.distributed as dist
    props = torch.cuda.get_device_properties(local)
    me = {"rank": rank, "local_rank": local, "device": local, "name": props.name,
          "pci_bus_id": getattr(props, "pci_bus_id", None), "uuid": str(getattr(props, "uuid", "")),
          "timed_s": elapsed}
    if world > 1 and dist.is_initialized():
        allr = [None] * dist.get_world_size()
        dist.all_gather_object(allr, me)
        return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()), "per_rank": allr}
    return {"world_size": 1, "backend": None, "per_rank": [me]}


# MI355X (MI355X_MICROARCH.md): 8 TB/s HBM3E; 256 CUs x 4 SIMD-32 at 2.4 GHz peak engine clock; a wave64 VALU
# instruction takes 2 SIMD cycles; the LDS array of each CU runs one cycle per clock.
HBM_PEAK_GBPS = 8000.0
CLOCK_HZ = 2.4e9
VALU_PEAK = 1024 * CLOCK_HZ / 2 / 1e9      # G wave64-VALU instructions / s
LDS_PEAK = 256 * CLOCK_HZ / 1e9            # G LDS-array cycles / s (all CUs)


def roofline(n, E, B, launch_ms, args, kpath):
    """The decode launch against the resource that binds it.

    * Streaming (generic CSR) kernels move every message through HBM each iteration: bound "hbm",
      achieved = SURVEY §8(d) algorithmic bytes per launch / launch time.
    * The register-resident QC kernels keep all messages on chip (HBM sees only llr in / bits out), so
      HBM cannot bind them: bound = the busier of VALU issue and the LDS pipe (ds_bpermute lane
      rotations), from the per-launch instruction / LDS-cycle counts that scripts/gpu_profile.sh measured
      for this exact configuration (profiles/counters.json; deterministic for a fixed iteration count; for
      early stop they depend on the data, so the record must also have this Eb/N0 grid and seed)
      divided by this run's event-timed launch duration, against 2.4 GHz peak.  The survey's byte model
      is kept beside it as hbm.model_frac (it exceeds 1 for on-chip kernels by construction) with the
      measured PMC traffic.
    """
    s_b = 1 if args.algo in ("qminsum", "qms") else 4  # 5-bit mode s_m = s_L = 1 byte
    bpc = algorithmic_bytes_per_cw(n, E, args.iters, s_b, s_b)
    launch_s = launch_ms * 1e-3
    model_gbps = bpc * B / launch_s / 1e9
    rec = None
    note = None
    if os.path.exists(args.counters_json):
        want = {"code": args.code, "algo": args.algo, "iters": args.iters, "early_stop": args.early_stop,
                "batch_per_gpu": B, "kernel_path": kpath, "mod": args.mod}
        if args.early_stop:  # the work done depends on the data (iterations to convergence): same grid and seed
            want.update(ebn0=args.ebn0, seed=args.seed)
        for r in json.load(open(args.counters_json)):
            if all(r["config"].get(k) == v for k, v in want.items()):
                rec = r
        if rec is None and args.early_stop:
            note = "no counter record for this Eb/N0 grid and seed (early-stop work depends on the data)"
    c = rec["counters_per_launch"] if rec else {}
    hbm_bytes = rec["derived"].get("hbm_bytes") if rec else None
    hbm = {"model_bytes_per_codeword": bpc, "model_GBps": model_gbps, "model_frac": model_gbps / HBM_PEAK_GBPS,
           "traffic_bytes_per_launch": hbm_bytes,
           "traffic_GBps": hbm_bytes / launch_s / 1e9 if hbm_bytes else None,
           "traffic_frac": hbm_bytes / launch_s / 1e9 / HBM_PEAK_GBPS if hbm_bytes else None}
    out = {"launch_ms": launch_ms, "hbm": hbm,
           "counters": (os.path.relpath(args.counters_json, ROOT) + f" [{rec['name']}]") if rec else note}
    if kpath == "generic-csr" or "SQ_INSTS_VALU" not in c:
        out.update(bound="hbm", achieved=model_gbps, peak=HBM_PEAK_GBPS, unit="GB/s",
                   frac=model_gbps / HBM_PEAK_GBPS, traffic=hbm_bytes)
        return out
    valu = c["SQ_INSTS_VALU"] / launch_s / 1e9
    lds = c.get("SQ_LDS_IDX_ACTIVE", 0.0) / launch_s / 1e9
    out["valu"] = {"achieved": valu, "peak": VALU_PEAK, "unit": "G wave-instr/s", "frac": valu / VALU_PEAK,
                   "insts_per_launch": c["SQ_INSTS_VALU"]}
    out["lds"] = {"achieved": lds, "peak": LDS_PEAK, "unit": "G LDS-cycles/s", "frac": lds / LDS_PEAK,
                  "cycles_per_launch": c.get("SQ_LDS_IDX_ACTIVE")}
    b = "lds" if out["lds"]["frac"] > out["valu"]["frac"] else "valu"
    out.update(bound=b, achieved=out[b]["achieved"], peak=out[b]["peak"], unit=out[b]["unit"], frac=out[b]["frac"],
               traffic=hbm_bytes)
    return out


def side_measurements(H, dec, llr_dev, B, args):
    """Two secondary numbers next to the headline (never `value`):
    * ``dropin``: the reference's boundary itself, ``decode_bits(llrs_f64, H, iters, 256, 10)``
      (ofdm_functions.py:131-163) from host float64 LLRs to host float64 bits — PCIe, staging and the
      f64<->f32 conversions included (ldpc_decode_bits_host's pinned two-stream pipeline);
    * ``gpu_tanh_sp``: the reference's algorithm (tanh sum-product, 50 it, clamp 10) on the same H with
      LLRs resident in HBM — the apples-to-apples partner of the reference CPU number."""
    import torch
    import ldpc_amd
    from ldpc_amd import _abi
    lib = _abi.load()
    host = llr_dev.double().cpu().numpy()
    # graph + staging ring at this size; two calls reach the steady state of a caller's loop
    # (`bits = decode_bits(...)` per SNR point: two output buffers alternate, api._OutputPool)
    for _ in range(2):
        out = ldpc_amd.decode_bits(host, H, args.iters, 256, 10.0)
    reps = 3
    t = time.perf_counter()
    for _ in range(reps):
        out = ldpc_amd.decode_bits(host, H, args.iters, 256, 10.0)   # a new float64 result each call, as the reference
    dt = (time.perf_counter() - t) / reps
    dropin = {"cw_per_s": B / dt, "seconds": dt, "codewords": B, "iters": args.iters, "algo": "tanh",
              "clamp": 10.0, "batch_size": 256, "bits_set": int(out.sum()),
              "what": "decode_bits(llrs float64 host, H, iters, 256, 10) end to end: f64->f32 staging, "
                      "H2D, decode, D2H, 0/1 float64 expansion"}
    p = dec.params(args.iters, "tanh", 10.0, device_ptrs=True)
    wsb = dec.workspace_bytes(B, p)
    ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=llr_dev.device)
    bits = torch.empty((B, dec.n), dtype=torch.uint8, device=llr_dev.device)
    st = torch.cuda.current_stream().cuda_stream
    run = lambda: _abi.check(lib.ldpc_decode_ex(dec._h, llr_dev.data_ptr(), B, p, bits.data_ptr(), None, None,
                                                ws.data_ptr(), wsb, st))
    run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    steps = 3
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    return {"dropin": dropin,
            "gpu_tanh_sp": {"cw_per_s": B / dt, "ms_per_launch": dt * 1e3, "codewords": B, "iters": args.iters,
                            "clamp": 10.0, "what": "tanh sum-product (the reference's algorithm), LLRs in HBM"}}


def reference_cpu(args):
    """The reference's own CPU path, timed in the build container by scripts/time_reference_cpu.py (the
    reference cannot travel to the GPU box); carried here with its provenance."""
    if args.code != "wifi648_12":
        return None
    if not os.path.exists(args.ref_cpu_json):  # never silently dropped (the box must carry the record)
        return {"missing": os.path.relpath(args.ref_cpu_json, ROOT), "kind": "reference"}
    r = json.load(open(args.ref_cpu_json))
    return {"value": r["reference_cw_per_s"], "unit": "codewords/s", "cores": r["threads"], "kind": "reference",
            "sample": f"{r['codewords']} codewords, decode_bits(llrs, H, {r['iters']}, {r['batch_size']}, "
                      f"{r['clamp']:g}) tanh-SP on the real (648,1/2) H at Eb/N0 {r['ebn0_db']} dB, "
                      f"{r['reference_seconds']:.1f} s, torch {r['torch']} CPU, {r['threads']} threads",
            "where": "build container (8-core Xeon, no GPU): " + os.path.relpath(args.ref_cpu_json, ROOT),
            "algo": "tanh", "iters": r["iters"]}


def cpu_baseline(H, args, rate):
    """The CPU oracle (oracle/ldpc_oracle.c, OpenMP over codewords) on a bounded sample of the same
    workload: same code, algorithm and iteration count, Eb/N0 = 2.5 dB.  CPU comparator only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from ldpc_amd.codes import Encoder, IRAEncoder, SparseCode
    rng = np.random.default_rng(5)
    enc = IRAEncoder(H) if isinstance(H, SparseCode) else Encoder(H)

    def sample(Bs):
        c = enc.encode(rng.integers(0, 2, size=(Bs, enc.k)))
        sigma = np.sqrt(1.0 / (2 * rate * 10 ** (2.5 / 10)))
        return (-2.0 * ((1.0 - 2.0 * c) + sigma * rng.standard_normal(c.shape)) / sigma**2).astype(np.float32)

    def run(x):
        t = time.perf_counter()
        if args.algo in ("minsum", "ms", "min_sum"):
            oracle.ms_f32(H, x, args.iters, args.clamp, args.alpha, 0.0, early_stop=args.early_stop)
        elif args.algo in ("qminsum", "qms"):
            q = np.clip(np.rint(x / args.qstep), -15, 15).astype(np.int8)
            oracle.qms(H, q, args.iters, early_stop=args.early_stop)
        else:
            oracle.sp_f32(H, x, args.iters, args.clamp, early_stop=args.early_stop, stable=True)
        return time.perf_counter() - t

    threads = oracle.num_threads()
    cal = max(64, 8 * threads)
    tc = run(sample(cal))
    Bs = int(min(1 << 17, max(cal, cal * args.cpu_seconds / max(tc, 1e-6))))
    t = run(sample(Bs))
    return {"value": Bs / t, "unit": "codewords/s", "cores": threads, "kind": "port",
            "sample": f"{Bs} codewords of {args.code} {args.algo} {args.iters} iters"
                      f"{' early-stop' if args.early_stop else ''} at Eb/N0 2.5 dB "
                      f"({t:.1f} s, oracle/ldpc_oracle.c, OpenMP {threads} threads)"}


if __name__ == "__main__":
    main()
