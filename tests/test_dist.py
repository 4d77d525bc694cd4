"""Multi-process (gloo, world_size 2) coverage of the sharded sweep: the same code path bench.py runs
with backend nccl (RCCL) on GPUs, here with a CPU decoder (the oracle, as test infrastructure)."""
import multiprocessing as mp
import socket

import numpy as np
import pytest

from dist_worker import POINTS, TOTAL, _run_shard_factory, _worker
from ldpc_amd.codes import Encoder, get_code
from ldpc_amd.dist import ebn0_sigma, shard_bounds, sweep

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_exactly():
    for total in (0, 1, 7, 64, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def test_sigma_formula():
    assert abs(ebn0_sigma(0.0, 0.5) - 1.0) < 1e-12


def test_two_rank_gloo_sweep_equals_single_process():
    H, _ = get_code("peg64_32")
    enc = Encoder(H)
    single = sweep(POINTS, TOTAL, 0.5, enc.k, _run_shard_factory(H, enc))
    ctx = mp.get_context("spawn")  # fork after libgomp started its pool deadlocks
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == out[1] == single.counts.tolist()
    assert single.counts[:, 2].tolist() == [TOTAL] * len(POINTS)
