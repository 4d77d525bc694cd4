#!/usr/bin/env python3
"""Headline benchmark: decoded codewords/s + BER vs Eb/N0, 802.11n (648,1/2), min-sum, 50 iterations.

One step = one decode of a batch of B = 65,536 codewords (per GPU) of one Eb/N0 point, LLRs already
resident in HBM; steps cycle through the 11 points Eb/N0 = 0:0.5:5 dB (BASELINE.json configs[1]).
Before timing, one untimed pass over all 11 points produces the BER/BLER curve (error counts on device,
summed over ranks with an RCCL all-reduce — the only collective; the codeword batches shard with no
data-path exchange, so scaling is weak).

    python bench.py [--gpus N --steps K --warmup W]                  # N ranks, one GPU each (started here)
    torchrun --nproc-per-node N ... bench.py --gpus N ...            # the same under a launcher

--gpus N is authoritative: without launcher variables, N > 1 starts N fresh rank processes of this script
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, RCCL) before this process touches a GPU, streams rank 0's
line and exits with the worst rank's code; under a launcher, WORLD_SIZE must equal N.

The other BASELINE.json configs run as short legs of the same script after the headline, reported under
``side.configs`` (never ``value``), each event-timed over LEGS[...]['passes'] launches per Eb/N0 point with its own
roofline from profiles/counters.json: configs[2] (1944,5/6) tanh-SP 50 it on 16-QAM OFDM LLRs, B=32,768;
configs[3] (1296,2/3) 5-bit min-sum <=20 it early stop, B=65,536; configs[4] DVB-S2 64800 rate 1/2 min-sum
50 it, B=4,096 per GPU.  Under torchrun (N>1) the config [4] leg runs on every rank — the BASELINE
multi-GPU configuration — with its counters summed by the same all-reduce and max-over-ranks timing.
Any of them alone: e.g. ``--code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768``.
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


def _dist_module():
    """ldpc_amd/dist.py loaded on its own: the launcher must not import the package (which loads the HIP
    library) before it has decided whether this process decodes or only starts the rank processes."""
    import importlib.util
    name = "_ldpc_amd_dist_launcher"
    if name not in sys.modules:
        spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "ldpc-sims_amd", "ldpc_amd", "dist.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
    return sys.modules[name]


def algorithmic_bytes_per_cw(n, E, iters, s_m=4, s_l=4):
    """the reference's two-array flooding dataflow per codeword:
    iters*(4*E*s_m + n*s_L) + n*s_L + n."""
    return iters * (4 * E * s_m + n * s_l) + n * s_l + n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 330 timed launches (30 passes over the 11 points, ~0.5 s): after the barrier / synchronize that open the
    # timed loop the engine clock needs ~8 launches to recover, 4-5 % of a 22-launch loop
    ap.add_argument("--steps", type=int, default=330)
    ap.add_argument("--warmup", type=int, default=11)
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
    ap.add_argument("--no-legs", action="store_true", help="skip the BASELINE configs[2..4] legs (side.configs)")
    ap.add_argument("--legs", default="auto",
                    help="comma list of legs (config2,config3,config4); auto = all three at N=1, config4 at N>1")
    ap.add_argument("--leg-batch-scale", type=float, default=1.0, help=argparse.SUPPRESS)
    ap.add_argument("--ref-cpu-json", default=os.path.join(ROOT, "profiles", "ref_cpu_wifi648.json"),
                    help="the reference's own CPU decode_bits timing (scripts/time_reference_cpu.py)")
    ap.add_argument("--counters-json", default=os.path.join(ROOT, "profiles", "counters.json"),
                    help="per-launch PMC counts per configuration (scripts/gpu_profile.sh + counters_summary.py)")
    args = ap.parse_args()

    # --gpus N is authoritative: under a launcher (torchrun) WORLD_SIZE must equal N; without one, N > 1
    # starts N fresh rank processes of this script (one GPU each, RCCL) before this process touches a GPU
    launcher = _dist_module()
    spawn = launcher.resolve_world(args.gpus)
    if spawn is not None and spawn > 1:
        if not os.environ.get("LDPC_BENCH_SHARE_GPU"):
            import torch  # device_count() does not initialise the GPU (this process only starts children)
            have = torch.cuda.device_count()
            if have < spawn:
                raise SystemExit(f"--gpus {spawn} but only {have} GPU(s) visible")
        log(f"bench: starting {spawn} rank processes")
        sys.exit(launcher.spawn_ranks([os.path.abspath(__file__), *sys.argv[1:]], spawn))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LDPC_BENCH_BACKEND / device modulo exist only to rehearse N>1 on a 1-GPU box (ranks share cuda:0,
    # counters over gloo); the driver's multi-GPU runs use the defaults: one GPU per rank, RCCL.
    local = local % max(1, torch.cuda.device_count()) if os.environ.get("LDPC_BENCH_SHARE_GPU") else local
    torch.cuda.set_device(local)
    # LDPC_BENCH_PG=1: a process group even at world size 1 — the RCCL path (init, barriers, the rank gather)
    # on a 1-GPU box, where RCCL refuses two ranks on one device (tests/test_gpu_multirank.py)
    if world > 1 or os.environ.get("LDPC_BENCH_PG") == "1":
        backend = os.environ.get("LDPC_BENCH_BACKEND", "nccl")  # nccl == RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    wl = Workload(args, rank, local)
    pending = wl.ber_launch()           # untimed BER pass over every point, queued: the warmup follows it directly
    elapsed, my_elapsed, gpu_ms = wl.timed(args.steps, args.warmup, world)
    ber = wl.ber_finish(pending)
    B, n, E = wl.B, wl.n, wl.E
    total_cw = world * args.steps * B
    ranks = rank_evidence(world, rank, local, my_elapsed, wl.clock)
    value = total_cw / elapsed
    roof = roofline(n, E, B, gpu_ms, args, wl.kpath, wl.m, wl.mean_iters, clock=wl.clock)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # CPU baseline at N=1 only
        cpu = cpu_baseline(wl.H, args, wl.rate)
    side = {}
    if rank == 0 and world == 1 and not args.no_dropin and B * n * 8 <= (1 << 32):
        side = side_measurements(wl.H, wl.dec, wl.llrs, B, args, wl.kpath)
        ref = reference_cpu(args)
        if cpu is not None and ref is not None:
            if "value" in ref:
                ref["gpu_tanh_sp_over_reference"] = side["gpu_tanh_sp"]["cw_per_s"] / ref["value"]
                ref["dropin_over_reference"] = side["dropin"]["cw_per_s"] / ref["value"]
                ref["headline_over_reference"] = value / ref["value"]
            cpu["reference"] = ref
    wl.free()
    # BASELINE.json configs[2..4] (never `value`): at N=1 all three on this GPU; at N>1 config [4] (the
    # DVB-S2 multi-GPU config) on every rank, its counters reduced by the same all-reduce
    legs = (list(LEGS) if world == 1 else ["config4"]) if args.legs == "auto" else [x for x in args.legs.split(",") if x]
    legs = [] if args.no_legs else legs
    for x in legs:
        if x not in LEGS:
            raise SystemExit(f"unknown leg {x!r}; choose from {sorted(LEGS)}")
    if legs:
        side["configs"] = {name: run_leg(name, args, rank, local, world) for name in legs}

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
            "config": wl.config_dict(world),
            # engine clock / power over rank 0's timed loop (every rank's in ranks.per_rank[].clock): the
            # headline kernel runs below the other kernels' clock, so throughput is quoted with the clock it ran at
            "clock": wl.clock,
            "ranks": ranks,
            "roofline": roof,
            "cpu_baseline": cpu,
            "dropin_cw_per_s": side["dropin"]["cw_per_s"] if "dropin" in side else None,
            "side": side or None,
            "ber": ber,
        }
        if getattr(wl, "step_trace_ms", None) is not None:
            out["step_trace_ms"] = [round(x, 4) for x in wl.step_trace_ms]
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


# BASELINE.json configs[2..4], each one short event-timed leg of this script (side.configs; never `value`)
LEGS = {
    "config2": dict(code="wifi1944_56", algo="tanh", iters=50, batch=32768, mod="16qam-ofdm", ebn0="4:0.5:9",
                    early_stop=False, passes=4, warmup=11,
                    baseline="configs[2]: tanh sum-product, (1944,5/6), 16-QAM OFDM front end"),
    "config3": dict(code="wifi1296_23", algo="qminsum", iters=20, batch=65536, mod="bpsk", ebn0="0:0.5:5",
                    early_stop=True, qstep=1.0, passes=30, warmup=11,
                    baseline="configs[3]: 5-bit LLR min-sum, (1296,2/3), 20 iters early termination"),
    "config4": dict(code="dvbs2_12", algo="minsum", iters=50, batch=4096, mod="bpsk", ebn0="0:0.5:2",
                    early_stop=False, passes=2, warmup=1,
                    baseline="configs[4]: DVB-S2 64800 rate 1/2, 50 iters, batch sharded"),
}


def leg_args(name, args):
    """The bench arguments of one BASELINE leg: this run's defaults (seed, clamp, counters record) with the
    leg's code / algorithm / batch / front end / Eb/N0 grid."""
    import argparse as _ap
    d = dict(vars(args))
    d.update(force_generic=False, alpha=1.0, qstep=1.0, clamp=20.0)
    d.update({k: v for k, v in LEGS[name].items() if k not in ("baseline", "passes", "warmup")})
    if args.leg_batch_scale != 1.0:  # tests only: a smaller batch (counter records then do not match)
        d["batch"] = max(64, int(d["batch"] * args.leg_batch_scale))
    return _ap.Namespace(**d)


def run_leg(name, args, rank, local, world):
    """One BASELINE config as a side leg: data resident in HBM, an untimed BER pass over its grid, the leg's
    warmup launches, then `passes` launches per Eb/N0 point event-timed (so an early-stop leg's mean launch is the
    sweep's mean; passes sized for a timed loop of >= ~0.3 s, past the clock ramp after the pre-loop
    synchronisation), max over ranks; roofline from this leg's own counter record."""
    import torch
    la = leg_args(name, args)
    wl = Workload(la, rank, local)
    pending = wl.ber_launch()
    P = len(wl.ebn0)
    steps = LEGS[name]["passes"] * P
    warm = LEGS[name]["warmup"]
    elapsed, my_elapsed, gpu_ms = wl.timed(steps, warm, world)
    ber = wl.ber_finish(pending)
    rec = {"baseline_config": LEGS[name]["baseline"], "value": world * steps * wl.B / elapsed,
           "unit": "codewords/s", "n_gpus": world, "steps": steps, "warmup": warm,
           "ms_per_step": elapsed / steps * 1e3, "ms_per_launch": gpu_ms,
           "config": wl.config_dict(world), "roofline": roofline(wl.n, wl.E, wl.B, gpu_ms, la, wl.kpath, wl.m, wl.mean_iters, clock=wl.clock),
           "mean_iters": wl.mean_iters, "clock": wl.clock, "ber": ber}
    if world > 1:
        rec["ranks"] = rank_evidence(world, rank, local, my_elapsed, wl.clock)
    wl.free()
    del wl
    torch.cuda.empty_cache()
    return rec


class Workload:
    """One bench configuration on this rank's GPU: the graph, synthetic LLRs for every Eb/N0 point resident
    in HBM (generated on device from the global codeword index, so the union of the ranks' shards is
    independent of the world size), decode parameters, workspace and output."""

    def __init__(self, args, rank, local):
        import torch
        import ldpc_amd
        from ldpc_amd import _abi
        from ldpc_amd.synth import DeviceEncoder
        self.args, self.rank = args, rank
        self.H, _ = ldpc_amd.get_code(args.code)
        m, n = self.H.shape
        self.m, self.n, self.k = m, n, n - m
        self.rate = self.k / n
        self.E = int(self.H.sum())  # nnz (SparseCode.sum() too)
        self.dec = ldpc_amd.get_decoder(self.H, local)
        B = self.B = args.batch
        lo, step_db, hi = (float(x) for x in args.ebn0.split(":"))
        self.ebn0 = np.round(np.arange(lo, hi + 1e-9, step_db), 6)
        self.lib = lib = _abi.load()
        self.stream = torch.cuda.current_stream()
        st = self.stream.cuda_stream
        enc = DeviceEncoder(self.H, torch.device("cuda", local))
        info = torch.empty((B, self.k), dtype=torch.uint8, device="cuda")
        _abi.check(lib.ldpc_random_bits(info.data_ptr(), B, self.k, args.seed, rank * B, st))
        self.cw = enc.encode(info)
        del info, enc
        self.llrs = []
        for i, e in enumerate(self.ebn0):
            x = torch.empty((B, n), dtype=torch.float32, device="cuda")
            if args.mod == "bpsk":
                sigma = float(np.sqrt(1.0 / (2.0 * self.rate * 10.0 ** (e / 10.0))))
                _abi.check(lib.ldpc_awgn_llr(self.cw.data_ptr(), x.data_ptr(), B, n, sigma, args.seed * 1000 + i,
                                             rank * B, st))
            else:
                from ldpc_amd.channel import ofdm_demod, ofdm_tx
                bps = 2 if args.mod == "qpsk-ofdm" else 4
                esn0 = float(10.0 ** (e / 10.0) * self.rate * bps)
                s_ = self.cw.view(-1)
                pad = (-s_.numel()) % (bps * 32)
                if pad:
                    s_ = torch.cat([s_, torch.zeros(pad, dtype=torch.uint8, device="cuda")])
                rx = ofdm_tx(s_, 32, bps, esn0, args.seed * 1000 + i, rank * B * n // bps)
                x.copy_(ofdm_demod(rx, 32, bps, esn0)[:B * n].view(B, n))
                del rx, s_
            self.llrs.append(x)
        self.p = self.dec.params(args.iters, args.algo, args.clamp, args.alpha, 0.0, args.early_stop, "f32", "p1",
                                 qstep=args.qstep, force_generic=args.force_generic, device_ptrs=True)
        self.kpath = self.dec.kernel_path(self.p)   # "qc-z<Z>", "ira-z360" or "generic-csr", as the library decides
        self.wsb = self.dec.workspace_bytes(B, self.p)
        self.ws = torch.empty((max(self.wsb, 1),), dtype=torch.uint8, device="cuda")
        self.bits = torch.empty((B, n), dtype=torch.uint8, device="cuda")

    def step(self, x, used=None):
        from ldpc_amd import _abi
        _abi.check(self.lib.ldpc_decode_ex(self.dec._h, x.data_ptr(), self.B, self.p, self.bits.data_ptr(), None,
                                           used.data_ptr() if used is not None else None, self.ws.data_ptr(), self.wsb,
                                           self.stream.cuda_stream))

    def ber(self):
        """Untimed pass over every point: error counts on device, summed over ranks (the one collective)."""
        return self.ber_finish(self.ber_launch())

    def ber_launch(self):
        """The BER pass's decodes and error counts, queued on the decode stream without a host synchronisation,
        so that the warmup and the timed loop follow them with no idle gap (DESIGN §5 "Timing window");
        ber_finish() reads the counts afterwards."""
        import torch
        from ldpc_amd import _abi
        from ldpc_amd.dist import allreduce_counts
        counts = torch.zeros((len(self.ebn0), 3), dtype=torch.int64, device="cuda")
        # with early stop, the iterations each codeword ran: their mean over the grid (the timed loop cycles over the
        # same points) is the byte model's iteration count
        used = torch.empty((self.B,), dtype=torch.int32, device="cuda") if self.args.early_stop else None
        used_sum = torch.zeros((), dtype=torch.int64, device="cuda")
        for i in range(len(self.ebn0)):
            self.step(self.llrs[i], used)
            if used is not None:
                used_sum += used.sum()
            _abi.check(self.lib.ldpc_count_errors(self.bits.data_ptr(), self.cw.data_ptr(), self.B, self.n, self.k,
                                                  counts[i].data_ptr(), self.stream.cuda_stream))
        return counts, used, used_sum

    def ber_finish(self, pending):
        from ldpc_amd.dist import allreduce_counts
        counts, used, used_sum = pending
        allreduce_counts(counts)  # 24 B x points per rank (RCCL)
        c = counts.cpu().numpy().astype(np.float64)
        self.mean_iters = (float(used_sum.item()) / (self.B * len(self.ebn0))) if used is not None else float(self.args.iters)
        return {"ebn0_db": self.ebn0.tolist(), "coded_ber_info": (c[:, 0] / (c[:, 2] * self.k)).tolist(),
                "coded_bler": (c[:, 1] / c[:, 2]).tolist(), "codewords_per_point": int(c[0, 2])}

    def timed(self, steps, warmup, world):
        """W untimed steps, then exactly K steps cycling over the points, bracketed by a barrier and a device
        synchronize on both sides.  Returns (max-over-ranks seconds, this rank's seconds, mean event-timed
        launch ms on the decode stream)."""
        import torch
        import torch.distributed as dist
        from ldpc_amd.dist import max_over_ranks
        from ldpc_amd.gpuclock import ClockSampler
        P = len(self.ebn0)
        # engine clock / power while the loop runs; built before the warmup so that amdsmi's start-up is not an
        # idle gap between the warmup and the timed loop (after an idle gap the engine clock ramps up again over
        # the first ~8 launches: DESIGN §5)
        sampler = ClockSampler(torch.cuda.current_device())
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        for w in range(warmup):
            self.step(self.llrs[w % P])
        # the sampler's first read and thread start happen while the warmup still runs, so that the only idle time
        # before the timed loop is the synchronisation itself; its samples are kept from t0 on
        with sampler:
            t0 = time.perf_counter()   # DIAGNOSTIC COPY: no synchronisation before the timed loop
            ev0.record(self.stream)
            trace = [] if os.environ.get("LDPC_BENCH_STEP_TRACE") else None   # diagnostic: one event per step
            for s in range(steps):
                if trace is not None:
                    trace.append(torch.cuda.Event(enable_timing=True))
                    trace[-1].record(self.stream)
                self.step(self.llrs[s % P])
            ev1.record(self.stream)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if dist.is_initialized():
                dist.barrier()
            # the closing synchronize and barrier are inside the bracket; the sampler's stop (a thread join of up to
            # one poll period and a last amdsmi read) is not: it had added ~0.7 ms to a 20-launch loop
            mine = time.perf_counter() - t0
        gpu_ms = ev0.elapsed_time(ev1) / max(steps, 1)
        if trace is not None:
            ends = trace[1:] + [ev1]
            self.step_trace_ms = [a.elapsed_time(b) for a, b in zip(trace, ends)]
        self.clock = sampler.summary(since=t0)
        self.clock["window_s"] = t1 - t0
        return max_over_ranks(mine, device="cuda"), mine, gpu_ms

    def config_dict(self, world):
        a = self.args
        return {"workload": f"{a.code} {a.algo} {a.iters} iters{' early-stop' if a.early_stop else ''}, "
                            f"B={self.B} codewords/GPU/step, Eb/N0 {a.ebn0} dB cycled per step",
                "code": a.code, "n": self.n, "k": self.k, "edges": self.E, "algo": a.algo, "iters": a.iters,
                "clamp": a.clamp, "alpha": a.alpha, "early_stop": a.early_stop, "mod": a.mod,
                "ebn0": a.ebn0, "seed": a.seed,
                "batch_per_gpu": self.B, "global_batch": self.B * world,
                "parallelism": f"dp{world} (codeword shards, RCCL all-reduce of error counts only)",
                "kernel_path": self.kpath,
                # the library's tuning knobs set in the environment (LDPC_*: chunk budget, streams, a variant
                # library, ...): empty for the shipped configuration; a counter record must match it
                "env": library_env()}

    def free(self):
        self.llrs = []
        self.cw = self.ws = self.bits = None


def library_env():
    """LDPC_* environment overrides of the library's defaults in this process (bench's own LDPC_BENCH_* launch knobs
    excluded: they place ranks, not kernels)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("LDPC_") and not k.startswith("LDPC_BENCH_")}


def rank_evidence(world, rank, local, elapsed, clock=None):
    """What the process group itself reports: world size and backend from torch.distributed, and every
    rank's device (index, name, PCI bus, UUID) and timed-region seconds, gathered to rank 0 over the same
    group (the counter all-reduce's), so a multi-GPU record shows that RCCL saw N ranks on N GPUs."""
    import torch
    import torch.distributed as dist
    props = torch.cuda.get_device_properties(local)
    me = {"rank": rank, "local_rank": local, "device": local, "name": props.name,
          "pci_bus_id": getattr(props, "pci_bus_id", None), "uuid": str(getattr(props, "uuid", "")),
          "timed_s": elapsed, "clock": clock}
    if dist.is_initialized():
        allr = [None] * dist.get_world_size()
        dist.all_gather_object(allr, me)
        return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()), "per_rank": allr}
    return {"world_size": 1, "backend": None, "per_rank": [me]}


# MI355X (MI355X_MICROARCH.md): 8 TB/s HBM3E; 256 CUs x 4 SIMD-32 at 2.4 GHz peak engine clock; a wave64 VALU
# instruction takes 2 SIMD cycles; the LDS array of each CU runs one cycle per clock.
HBM_PEAK_GBPS = 8000.0
IC_GATHER_GBPS = 8600.0   # Infinity Cache, uniformly gathered rows (MI355X_MICROARCH.md, "Indexed rows")
CLOCK_HZ = 2.4e9
VALU_PEAK = 1024 * CLOCK_HZ / 2 / 1e9      # G wave64-VALU instructions / s
LDS_PEAK = 256 * CLOCK_HZ / 1e9            # G LDS-array cycles / s (all CUs)


def ira_bytes_per_cw(n, m, iters):
    """Bytes per codeword the DVB-S2-structured min-sum kernels (csrc/ira.hip) move beyond L2: load (llr in,
    L out: 8n), state init (12m), iters + 1 VN passes (L in, check states in, app out: 8n + 12m each), iters CN
    passes (app in, states in and out: 4n + 24m each), output (app in, bits out: 5n)."""
    return iters * (12 * n + 36 * m) + 21 * n + 24 * m


def roofline(n, E, B, launch_ms, args, kpath, m=None, iters=None, clock=None):
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
    it = args.iters if iters is None else iters  # early stop: the mean iterations executed
    bpc = algorithmic_bytes_per_cw(n, E, it, s_b, s_b)
    launch_s = launch_ms * 1e-3
    model_gbps = bpc * B / launch_s / 1e9
    rec = None
    note = None
    if os.path.exists(args.counters_json):
        want = {"code": args.code, "algo": args.algo, "iters": args.iters, "early_stop": args.early_stop,
                "batch_per_gpu": B, "kernel_path": kpath, "mod": args.mod, "env": library_env()}
        if args.early_stop:  # the work done depends on the data (iterations to convergence): same grid and seed
            want.update(ebn0=args.ebn0, seed=args.seed)
        for r in json.load(open(args.counters_json)):
            if all(r["config"].get(k) == v for k, v in want.items()):
                rec = r
        if rec is None and args.early_stop:
            note = "no counter record for this Eb/N0 grid and seed (early-stop work depends on the data)"
    c = rec["counters_per_launch"] if rec else {}
    hbm_bytes = rec["derived"].get("hbm_bytes") if rec else None
    hbm = {"model_bytes_per_codeword": bpc, "model_iters": it, "model_GBps": model_gbps, "model_frac": model_gbps / HBM_PEAK_GBPS,
           "traffic_bytes_per_launch": hbm_bytes,
           "traffic_GBps": hbm_bytes / launch_s / 1e9 if hbm_bytes else None,
           "traffic_frac": hbm_bytes / launch_s / 1e9 / HBM_PEAK_GBPS if hbm_bytes else None}
    out = {"launch_ms": launch_ms, "hbm": hbm,
           "counters": (os.path.relpath(args.counters_json, ROOT) + f" [{rec['name']}]") if rec else note}
    if kpath == "ira-z360":
        # the kernel's own dataflow (compressed check states, posteriors): its bytes per codeword, not the
        # survey's two-array model (kept beside it as hbm.model_*, which this kernel exceeds by design)
        # These bytes leave L2 but are served mostly by the 256 MiB Infinity Cache (the decode runs in chunks
        # sized to it), and FETCH_SIZE/WRITE_SIZE count such hits too (MI355X_MICROARCH.md, HBM):
        # the yardstick is the memory side beyond L2, priced against the guide's Infinity-Cache gather rate
        # (8.6 TB/s), with the fraction of the 8 TB/s HBM peak beside it — a yardstick, not the binding limit
        # (bound_note: fewer bytes measured no faster).
        ib = ira_bytes_per_cw(n, m, it)
        own = ib * B / launch_s / 1e9
        out.update(bound="memory-side (beyond L2, Infinity Cache included)", achieved=own, peak=IC_GATHER_GBPS,
                   unit="GB/s", frac=own / IC_GATHER_GBPS, hbm_frac=own / HBM_PEAK_GBPS, traffic=hbm_bytes,
                   traffic_note="2*FETCH_SIZE + WRITE_SIZE per launch: memory-side requests, Infinity-Cache hits included",
                   bound_note="byte model as the yardstick; measured not byte-bound: 20 % fewer bytes per iteration "
                              "ran at the same speed (DESIGN.md 3.8, profiles/r06/ab/ab_c4_ira_r6x.txt)",
                   bytes_per_codeword=ib, bytes_model="ira: iters*(12n + 36m) + 21n + 24m (csrc/ira.hip)")
        return out
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
    mhz = (clock or {}).get("clock_mhz")
    if mhz:
        # the on-chip peaks scale with the engine clock: the same fraction against the peak at the mean clock the
        # timed loop ran at (a loaded chip runs below the 2.4 GHz the peak assumes)
        out["frac_at_clock"] = out["frac"] * CLOCK_HZ / (mhz * 1e6)
        out["clock_mhz"] = mhz
    return out


def side_measurements(H, dec, llrs, B, args, kpath):
    """Two secondary numbers next to the headline (never `value`):
    * ``dropin``: the reference's boundary itself, ``decode_bits(llrs_f64, H, iters, 256, 10)``
      (ofdm_functions.py:131-163) from host float64 LLRs to host float64 bits — PCIe, staging and the
      f64<->f32 conversions included (ldpc_decode_bits_host's pinned two-stream pipeline), at the
      middle Eb/N0 point;
    * ``gpu_tanh_sp``: the reference's algorithm (tanh sum-product, 50 it, clamp 10) on the same H with
      LLRs resident in HBM — the apples-to-apples partner of the reference CPU number.  Timed as the
      headline is: 3 warmup launches at size, then 2 launches per Eb/N0 point between two HIP events on
      the decode stream."""
    import torch
    import ldpc_amd
    from ldpc_amd import _abi
    lib = _abi.load()
    host = llrs[len(llrs) // 2].double().cpu().numpy()
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
    del host, out
    p = dec.params(args.iters, "tanh", 10.0, device_ptrs=True)
    wsb = dec.workspace_bytes(B, p)
    dev = llrs[0].device
    ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=dev)
    bits = torch.empty((B, dec.n), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    st = stream.cuda_stream

    def run(x):
        _abi.check(lib.ldpc_decode_ex(dec._h, x.data_ptr(), B, p, bits.data_ptr(), None, None, ws.data_ptr(), wsb, st))
    for w in range(3):
        run(llrs[w % len(llrs)])
    torch.cuda.synchronize()
    steps = 6 * len(llrs)   # ~0.25 s: past the clock ramp after the synchronize above
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for s in range(steps):
        run(llrs[s % len(llrs)])
    ev1.record(stream)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    import argparse as _ap
    targs = _ap.Namespace(**dict(vars(args), algo="tanh", clamp=10.0, early_stop=False))
    kpath = dec.kernel_path(p)
    return {"dropin": dropin,
            "gpu_tanh_sp": {"cw_per_s": B / (ms * 1e-3), "ms_per_launch": ms, "launches": steps, "warmup": 3,
                            "codewords": B, "iters": args.iters, "clamp": 10.0, "timing": "HIP events",
                            "what": "tanh sum-product (the reference's algorithm), LLRs in HBM",
                            "roofline": roofline(dec.n, dec.E, B, ms, targs, kpath, dec.m)}}


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
