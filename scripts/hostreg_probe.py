"""Probe (GPU box): cost of pinning a fresh 340 MB float64 host array in place (hipHostRegister) against
first-touch page faults and a pinned copy — for deciding whether the drop-in could DMA the caller's float64
LLRs and 0/1 output directly.  Prints JSON lines."""
import json
import time

import numpy as np
import torch

rt = torch.cuda.cudart()
B, n = 65536, 648
for rep in range(3):
    a = np.zeros((B, n))
    t0 = time.perf_counter()
    rc = rt.cudaHostRegister(a.ctypes.data, a.nbytes, 0)
    t1 = time.perf_counter()
    rt.cudaHostUnregister(a.ctypes.data)
    t2 = time.perf_counter()
    b = np.zeros((B, n))
    t3 = time.perf_counter()
    b[:] = 1.0
    t4 = time.perf_counter()
    a2 = np.ones((B, n))
    rt.cudaHostRegister(a2.ctypes.data, a2.nbytes, 0)
    d = torch.empty((B, n), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    d.copy_(torch.from_numpy(a2), non_blocking=True)
    torch.cuda.synchronize()
    t6 = time.perf_counter()
    torch.from_numpy(a2).copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    t7 = time.perf_counter()
    rt.cudaHostUnregister(a2.ctypes.data)
    print(json.dumps({"register_fresh_ms": (t1 - t0) * 1e3, "rc": int(rc), "unregister_ms": (t2 - t1) * 1e3,
                      "first_touch_ms": (t4 - t3) * 1e3, "h2d_registered_GBps": a2.nbytes / (t6 - t5) / 1e9,
                      "d2h_registered_GBps": a2.nbytes / (t7 - t6) / 1e9}), flush=True)
