#!/usr/bin/env python3
"""Time the REFERENCE's own CPU decode path on the real 802.11n (648,1/2) H (build container only).

The reference (/root/reference/pytorch) never travels to the GPU box, so its CPU throughput is measured
here, once, and committed as profiles/ref_cpu_wifi648.json; bench.py carries it in
``cpu_baseline.reference`` with this provenance.  What is timed is exactly what every reference evaluator
calls: ``decode_bits(llrs, H, 50, batch_size, clamp)`` (``pytorch/ofdm/ofdm_functions.py:131-163``), i.e.
``BeliefPropagation(H, 50)`` (tanh sum-product, ``bp/bp.py:20-51``) batch by batch, with torch's
intra-op threads = the cores stated.  The build's C oracle (same algorithm, OpenMP over codewords) runs on
the same LLRs and cores beside it, so the two CPU numbers are directly comparable.

    PYTHONDONTWRITEBYTECODE=1 python scripts/time_reference_cpu.py [--batch 64] [--batches 2] [--threads 8]
"""
import argparse
import json
import os
import platform
import sys
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/pytorch"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--batches", type=int, default=2)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--clamp", type=float, default=10.0)
    ap.add_argument("--ebn0", type=float, default=2.5)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "ref_cpu_wifi648.json"))
    a = ap.parse_args()

    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(ROOT, "ldpc-sims_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import torch
    np.complex = complex  # the reference uses np.complex/np.float (removed in numpy 2); in-process shim only
    np.float = float
    os.environ["OMP_NUM_THREADS"] = str(a.threads)   # before the oracle library loads
    torch.set_num_threads(a.threads)
    from ofdm import ofdm_functions as OF
    from ldpc_amd.codes import Encoder, get_code
    import oracle

    H, _ = get_code("wifi648_12")
    H = np.asarray(H, np.int64)
    enc = Encoder(H)
    rate = enc.k / H.shape[1]
    N = a.batch * a.batches
    rng = np.random.default_rng(648)
    cw = enc.encode(rng.integers(0, 2, size=(N, enc.k)))
    sigma2 = 1.0 / (2.0 * rate * 10.0 ** (a.ebn0 / 10.0))
    llr = (-2.0 * ((1.0 - 2.0 * cw) + np.sqrt(sigma2) * rng.standard_normal(cw.shape)) / sigma2)

    t = time.perf_counter()
    bits_ref = OF.decode_bits(llr, H, a.iters, a.batch, a.clamp)
    t_ref = time.perf_counter() - t

    t = time.perf_counter()
    bits_or = oracle.sp_f32(H, llr.astype(np.float32), a.iters, a.clamp)["bits"]
    t_or = time.perf_counter() - t
    agree = int((bits_or.astype(np.float64) == bits_ref).sum())

    rec = {
        "what": "reference decode_bits (pytorch/ofdm/ofdm_functions.py:131-163), tanh-SP BeliefPropagation "
                "(bp/bp.py:20-51), real 802.11n (648,1/2) H",
        "code": "wifi648_12", "n": int(H.shape[1]), "E": int(H.sum()), "iters": a.iters, "clamp": a.clamp,
        "ebn0_db": a.ebn0, "batch_size": a.batch, "codewords": N,
        "reference_seconds": t_ref, "reference_cw_per_s": N / t_ref,
        "oracle_tanh_sp_seconds": t_or, "oracle_tanh_sp_cw_per_s": N / t_or,
        "hard_bits_agree": f"{agree}/{bits_ref.size}",
        "bit_errors_vs_codeword": int((bits_ref != cw).sum()),
        "threads": a.threads, "oracle_threads": oracle.num_threads(), "cpu": platform.processor() or platform.machine(), "nproc": os.cpu_count(),
        "torch": torch.__version__, "numpy": np.__version__,
        "host": "build container (no GPU); the reference cannot run on the GPU box",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
