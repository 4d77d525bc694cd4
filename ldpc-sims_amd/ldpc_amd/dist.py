"""Multi-GPU BER/BLER sweep: one process per GPU, codeword shards, one collective per SNR sweep.

The reference's only parallelism is ``nn.DataParallel`` over the codeword batch
(``ofdm/ofdm_functions.py:141-145``): a single process scattering dim 0 to every GPU and gathering the
decoded bits back to GPU 0 each batch.  Here every rank owns its shard for the whole sweep: it
generates its own LLRs on device (counter-based channel keyed by the GLOBAL codeword index, so the
union of the shards is the same data whatever the world size), decodes, counts errors on device, and
the ranks exchange nothing but the error counters — ``int64[n_points][3] = {info bit errors, block
errors, codewords}`` — in one all-reduce (RCCL over xGMI with backend "nccl"; gloo on CPU in tests).
That matches the metrics of ``evaluate_quantized.py:139-141`` (coded BER over info bits, BLER over all
bits).  No data-path collective exists because decoding never exchanges messages between codewords.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import Callable, Sequence

import numpy as np


def shard_bounds(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of ``total`` codewords for ``rank``; sizes differ by at most one."""
    if world <= 0 or not (0 <= rank < world) or total < 0:
        raise ValueError("bad shard arguments")
    q, r = divmod(total, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def ebn0_sigma(ebn0_db: float, rate: float) -> float:
    """BPSK noise std for Eb/N0: sigma^2 = 1 / (2 R Eb/N0)."""
    return float(np.sqrt(1.0 / (2.0 * rate * 10.0 ** (ebn0_db / 10.0))))


@dataclass
class SweepResult:
    ebn0_db: list
    counts: np.ndarray        # (points, 3) int64 summed over ranks
    info_bits: int

    @property
    def coded_ber(self):
        return (self.counts[:, 0] / np.maximum(self.counts[:, 2] * self.info_bits, 1)).tolist()

    @property
    def coded_bler(self):
        return (self.counts[:, 1] / np.maximum(self.counts[:, 2], 1)).tolist()


def _backend_device_ok(t, group):
    import torch.distributed as dist
    # gloo reduces CPU tensors only: stage through host when the counters live on the GPU
    return not (t.is_cuda and dist.get_backend(group) == "gloo")


def allreduce_counts(counts, group=None):
    """Sum the per-point error counters over ranks (the only collective)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if _backend_device_ok(counts, group):
            dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
        else:
            h = counts.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            counts.copy_(h)
    return counts


def max_over_ranks(value: float, device="cpu", group=None) -> float:
    import torch
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.tensor([value], dtype=torch.float64, device=device)
        if not _backend_device_ok(t, group):
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return float(t.item())
    return value


RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def resolve_world(requested: int, env=None) -> int | None:
    """How a ``--gpus N`` entry point runs.  Returns None when this process is one rank of an existing
    launch (``WORLD_SIZE`` set, e.g. by torchrun or by ``spawn_ranks``) — then ``WORLD_SIZE`` must equal
    ``N`` or this raises ``SystemExit`` (a torchrun with a different rank count is a mislabelled run);
    otherwise returns N, the number of rank processes this process must start (1 = run in-process)."""
    env = os.environ if env is None else env
    if requested < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {requested})")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != requested:
            raise SystemExit(f"WORLD_SIZE={ws} from the launcher but --gpus {requested}: refusing a run whose "
                             "rank count differs from the one it would report")
        return None
    return requested


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(argv: Sequence[str], world: int, env=None, poll_s: float = 0.2) -> int:
    """Start ``world`` fresh child processes ``python <argv>`` — one rank per GPU, the environment torchrun
    would give them (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE, MASTER_ADDR 127.0.0.1 and a free
    port) — and wait for them.  The children inherit stdout / stderr, so rank 0's JSON line and every
    rank's progress stream through unchanged.  The caller must not have touched the GPU (it starts
    children, it never execs).  If any rank fails, the others are terminated (they would wait forever in
    a collective) and the worst return code is returned.

    This replaces the reference's single-process ``nn.DataParallel`` mode (ofdm_functions.py:141-145) with
    one process per GPU, so ``bench.py --gpus N`` runs N ranks without an external launcher."""
    env = dict(os.environ if env is None else env)
    for k in RANK_VARS:
        env.pop(k, None)
    port = _free_port()
    procs = []
    first = []   # return codes of the ranks that failed on their own (before any was terminated here)
    try:
        for r in range(world):
            e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                     MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, *argv], env=e))
        while True:
            rcs = [p.poll() for p in procs]
            first = [rc for rc in rcs if rc not in (None, 0)]
            if first or all(rc is not None for rc in rcs):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    rcs = [p.returncode for p in procs]
    bad = first or [rc for rc in rcs if rc != 0]
    if bad:
        print(f"spawn_ranks: rank return codes {rcs}", file=sys.stderr, flush=True)
        # a signal-killed child reports -signum: the shell's 128 + signum
        return max((128 - rc if rc < 0 else rc) for rc in bad)
    return 0


def sweep(points: Sequence[float], total_codewords: int, rate: float, info_bits: int,
          run_shard: Callable[[int, int, int, float], np.ndarray], rank: int = 0, world: int = 1,
          device="cpu", group=None) -> SweepResult:
    """Run a BER sweep sharded over ranks.

    ``run_shard(point_index, lo, hi, sigma)`` decodes the global codewords [lo, hi) at one point and
    returns that shard's ``int64[3]`` counters.  The GPU implementation (bench.py / sweep CLI) generates
    LLRs with ``ldpc_awgn_llr(..., b0=lo)`` and counts with ``ldpc_count_errors``; tests pass a CPU
    decoder.  Returns the world-summed counters.
    """
    import torch
    lo, hi = shard_bounds(total_codewords, rank, world)
    counts = torch.zeros((len(points), 3), dtype=torch.int64, device=device)
    for i, e in enumerate(points):
        if hi > lo:
            c = run_shard(i, lo, hi, ebn0_sigma(e, rate))
            counts[i] += torch.as_tensor(np.asarray(c, dtype=np.int64), device=device)
    allreduce_counts(counts, group)
    return SweepResult(list(points), counts.cpu().numpy(), info_bits)
