#!/usr/bin/env python3
"""Drop-in decode_bits (ldpc_decode_bits_host) end to end on (648,1/2), tanh-SP 50 it, 65,536 codewords from
host float64, over staging thread counts and chunk sizes (measure above 16 threads).  GPU box.

    python scripts/dropin_threads.py > gpurun_out/dropin_threads.jsonl
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ldpc-sims_amd"))


def main():
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import ldpc_amd
    from ldpc_amd import _abi
    H, _ = ldpc_amd.get_code("wifi648_12")
    B, n = 65536, H.shape[1]
    rng = np.random.default_rng(1)
    sigma = np.sqrt(1.0 / (2 * 0.5 * 10 ** (2.5 / 10)))
    llr = np.ascontiguousarray(-2.0 * (1.0 + sigma * rng.standard_normal((B, n))) / sigma**2)
    out = np.zeros((B, n))
    dec = ldpc_amd.get_decoder(H)
    p = dec.params(50, "tanh", 10.0)
    # the drop-in itself (fresh np.zeros output per call, as the reference's decode_bits), steady state
    for what, keep in (("decode_bits, result dropped each call", False), ("decode_bits, bits = ... loop", True)):
        r = None
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            x = ldpc_amd.decode_bits(llr, H, 50, 256, 10.0)
            ts.append(time.perf_counter() - t)
            r = x if keep else None
            del x
        print(json.dumps({"what": what, "times_s": ts, "cw_per_s_last3": B / (sum(ts[2:]) / 3)}), flush=True)
    for threads in (1, 4, 8, 12, 16, 24, 32):
        for chunk in (0, 2048, 16384):
            _abi.check(dec.lib.ldpc_decode_bits_host(dec._h, llr.ctypes.data, B, ctypes.byref(p), out.ctypes.data,
                                                     chunk, threads))
            ts = []
            for _ in range(3):
                t = time.perf_counter()
                _abi.check(dec.lib.ldpc_decode_bits_host(dec._h, llr.ctypes.data, B, ctypes.byref(p),
                                                         out.ctypes.data, chunk, threads))
                ts.append(time.perf_counter() - t)
            print(json.dumps({"threads": threads, "chunk": chunk, "best_s": min(ts), "cw_per_s": B / min(ts),
                              "cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}), flush=True)


if __name__ == "__main__":
    main()
