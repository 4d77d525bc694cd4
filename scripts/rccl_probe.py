#!/usr/bin/env python3
"""Probe: can torch.distributed's "nccl" backend (RCCL) run WORLD ranks on one GPU of this box?  Each rank is a
fresh child process (never exec); every rank all-reduces a device tensor of ones and prints the sum.
    python scripts/rccl_probe.py WORLD
"""
import os
import socket
import subprocess
import sys


def child():
    import torch
    import torch.distributed as dist
    r = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.ones(4, device="cuda") * (r + 1)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print("rank", r, "of", dist.get_world_size(), "backend", dist.get_backend(), "sum", t.tolist(), flush=True)
    dist.destroy_process_group()


def main():
    if os.environ.get("RCCL_PROBE_CHILD"):
        return child()
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), RCCL_PROBE_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    rc = 0
    for p in procs:
        try:
            rc |= p.wait(timeout=90)
        except subprocess.TimeoutExpired:
            p.kill()
            rc |= 124
    print("exit", rc)
    sys.exit(rc)


if __name__ == "__main__":
    main()
