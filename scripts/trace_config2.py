#!/usr/bin/env python3
"""Config [2] soft parity, traced: which operation separates the GPU's z from its
specification (the C oracle's (D, S) form) on the codewords that converge late in a 50-iteration (1944,5/6)
tanh-SP decode of 16-QAM OFDM LLRs — the failing case of round 4 (6.0 dB, seed 100, tests/test_gpu_config2.py).

For the library at LDPC_LIB (default: the in-tree build; the DS_CR diagnostic variants evaluate exp2, S/D and
log2 correctly rounded through fp64 — common.h) it records, for every decoded codeword of the batch:
  * conv_at: the iteration the oracle's early stop would have stopped at,
  * z after k = 1..50 iterations from the GPU, the oracle (D, S) fp32 and the fp64 target (oracle.sp_f64 with
    the fp32 module's p-clamp bound, pinned to the reference's .double() module in test_oracle_golden.py),
  * the first iteration at which the GPU's z differs from the oracle's (bitwise), and the errors vs fp64 at 50.
Writes one JSON object to stdout.

    LDPC_LIB=build_variants/cr7.so python scripts/trace_config2.py --label cr7 > gpurun_out/trace_c2_cr7.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("ldpc-sims_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="shipped")
    ap.add_argument("--ebn0", type=float, default=6.0)
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--trace-rows", type=int, default=12, help="late codewords traced per iteration")
    a = ap.parse_args()
    import torch
    import oracle
    import ldpc_amd
    from ldpc_amd.codes import Graph, get_code
    from test_gpu_config2 import _qam16_llrs
    H, _ = get_code("wifi1944_56")
    seed = 40 + int(a.ebn0 * 10)
    cw, x = _qam16_llrs(H, a.B, a.ebn0, seed=seed)
    dec = ldpc_amd.get_decoder(H)
    llr = x.cpu().numpy()
    r50 = dec.decode(x, 50, algo="tanh", clamp=20.0, soft="z")
    z50 = r50["soft"].cpu().numpy()
    ref = oracle.sp_f32(H, llr, 50, 20.0, stable=True)
    conv_at = oracle.sp_f32(H, llr, 50, 20.0, stable=True, early_stop=True)["iters_used"]
    t64 = oracle.sp_f64(H, llr.astype(np.float64), 50, 20.0, ceiling="f32")["z"]
    g = Graph.from_H(H)
    par = np.add.reduceat(ref["bits"][:, g.col_idx].astype(np.int64), g.row_ptr[:-1], axis=1) % 2
    ok = ~par.any(axis=1)
    scale = np.maximum(1.0, np.abs(t64))
    rel_gpu = (np.abs(z50 - t64) / scale).max(axis=1)
    rel_ora = (np.abs(ref["z"] - t64) / scale).max(axis=1)
    late = np.flatnonzero(ok & (conv_at > 40))
    early = np.flatnonzero(ok & (conv_at <= 40))
    out = {"label": a.label, "lib": os.environ.get("LDPC_LIB", "in-tree"), "ebn0": a.ebn0, "seed": seed,
           "B": a.B, "decoded": int(ok.sum()), "converged_by_40": int(len(early)), "converged_after_40": int(len(late)),
           "gpu_vs_f64_max_by_40": float(rel_gpu[early].max()) if len(early) else 0.0,
           "gpu_vs_f64_max_after_40": float(rel_gpu[late].max()) if len(late) else 0.0,
           "oracle_vs_f64_max_by_40": float(rel_ora[early].max()) if len(early) else 0.0,
           "oracle_vs_f64_max_after_40": float(rel_ora[late].max()) if len(late) else 0.0,
           "gpu_eq_oracle_bitwise_rows": int((z50.view(np.uint32) == ref["z"].view(np.uint32)).all(axis=1).sum()),
           "gpu_eq_oracle_bitwise_entries_frac": float((z50.view(np.uint32) == ref["z"].view(np.uint32)).mean()),
           "rows": []}
    rows = late[: a.trace_rows]
    if len(rows):
        xs = x[torch.from_numpy(rows).cuda()]
        lr = llr[rows]
        gz, oz, fz = [], [], []
        for k in range(1, 51):
            gz.append(dec.decode(xs, k, algo="tanh", clamp=20.0, soft="z")["soft"].cpu().numpy())
            oz.append(oracle.sp_f32(H, lr, k, 20.0, stable=True)["z"])
            fz.append(oracle.sp_f64(H, lr.astype(np.float64), k, 20.0, ceiling="f32")["z"])
        gz, oz, fz = np.stack(gz), np.stack(oz), np.stack(fz)          # (50, rows, n)
        sc = np.maximum(1.0, np.abs(fz))
        for j, rr in enumerate(rows):
            diff = (gz[:, j].view(np.uint32) != oz[:, j].view(np.uint32)).any(axis=1)
            first = int(np.argmax(diff)) + 1 if diff.any() else None
            out["rows"].append({
                "row": int(rr), "conv_at": int(conv_at[rr]), "first_gpu_ne_oracle_iter": first,
                "gpu_ne_oracle_entries_at_first": int((gz[first - 1, j].view(np.uint32) != oz[first - 1, j].view(np.uint32)).sum()) if first else 0,
                "gpu_vs_oracle_rel_by_iter": [float(v) for v in (np.abs(gz[:, j] - oz[:, j]) / sc[:, j]).max(axis=1)],
                "gpu_vs_f64_rel_by_iter": [float(v) for v in (np.abs(gz[:, j] - fz[:, j]) / sc[:, j]).max(axis=1)],
                "oracle_vs_f64_rel_by_iter": [float(v) for v in (np.abs(oz[:, j] - fz[:, j]) / sc[:, j]).max(axis=1)],
            })
    print(json.dumps(out))


if __name__ == "__main__":
    main()
