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
