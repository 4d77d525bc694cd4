"""Child of tests/test_launcher.py: one rank started by ldpc_amd.dist.spawn_ranks.  Joins a gloo group
from the environment the launcher set, all-reduces its rank, and rank 0 prints one JSON line.
``--fail-rank r`` makes rank r exit with code 3 before the collective (the others would then block in it)."""
import argparse
import json
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--fail-rank", type=int, default=-1)
a = ap.parse_args()
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
if rank == a.fail_rank:
    sys.exit(3)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

dist.init_process_group("gloo")
t = torch.tensor([rank + 1], dtype=torch.int64)
dist.all_reduce(t)
if rank == 0:
    print(json.dumps({"world": dist.get_world_size(), "sum": int(t.item()), "local": os.environ["LOCAL_RANK"],
                      "addr": os.environ["MASTER_ADDR"]}), flush=True)
dist.destroy_process_group()
