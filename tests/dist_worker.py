"""Worker for tests/test_dist.py (spawned processes import it by name).  Test infrastructure."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "ldpc-sims_amd"), os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from ldpc_amd.codes import Encoder, get_code  # noqa: E402
from ldpc_amd.dist import sweep  # noqa: E402

POINTS = [1.0, 2.0, 3.0]
TOTAL = 48


def _run_shard_factory(H, enc):
    def run_shard(i, lo, hi, sigma):
        # per-codeword RNG keyed by the GLOBAL index: shard-independent data (as ldpc_awgn_llr's b0)
        cws, llrs = [], []
        for b in range(lo, hi):
            rng = np.random.default_rng([77, i, b])
            c = enc.encode(rng.integers(0, 2, size=(1, enc.k)))[0]
            y = (1.0 - 2.0 * c) + sigma * rng.standard_normal(c.shape)
            cws.append(c)
            llrs.append((-2.0 * y / sigma**2).astype(np.float32))
        cw, llr = np.array(cws), np.array(llrs)
        bits = oracle.ms_f32(H, llr, 10, 20.0)["bits"]
        return [int((bits[:, :enc.k] != cw[:, :enc.k]).sum()), int((bits != cw).any(1).sum()), hi - lo]
    return run_shard


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H, _ = get_code("peg64_32")
    enc = Encoder(H)
    res = sweep(POINTS, TOTAL, 0.5, enc.k, _run_shard_factory(H, enc), rank=rank, world=world)
    q.put((rank, res.counts.tolist()))
    dist.destroy_process_group()


