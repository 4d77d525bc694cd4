#!/usr/bin/env python3
"""GPU half of scripts/trace_failure.py: z of every codeword of the (648,1/2) 50-iteration golden set (tag snr1)
after k = 1 .. 50 tanh-SP iterations (clamp 10; flooding, so k iterations = the first k of a 50-iteration run),
through the register kernel and the generic CSR kernels (asserted bitwise equal).  Writes gpurun_out/trace_gpu.npz.

    python scripts/trace_failure_gpu.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ldpc-sims_amd"))


def main():
    import torch
    import ldpc_amd
    from ldpc_amd.codes import qc_expand
    tag = sys.argv[1] if len(sys.argv) > 1 else "snr1"
    d = np.load(os.path.join(ROOT, "tests", "golden", "bp_wifi648_12_sp_it50.npz"))
    H = qc_expand(d["base"], int(d["Z"]))
    dec = ldpc_amd.get_decoder(H)
    x = torch.from_numpy(d[f"llr_{tag}"]).cuda()
    zs = []
    for k in range(1, int(d["iters"]) + 1):
        a = dec.decode(x, k, algo="tanh", clamp=float(d["clamp"]), soft="z")["soft"]
        b = dec.decode(x, k, algo="tanh", clamp=float(d["clamp"]), soft="z", force_generic=True)["soft"]
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), k
        zs.append(a.cpu().numpy())
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "trace_gpu.npz"), z=np.stack(zs), tag=tag)
    print("trace_gpu.npz", np.stack(zs).shape)


if __name__ == "__main__":
    main()
