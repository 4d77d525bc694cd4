#!/usr/bin/env python3
"""Iteration-by-iteration trace of the soft outputs on the (648,1/2) 50-iteration golden set at 1 dB
(tests/golden/bp_wifi648_12_sp_it50.npz, snr1), where the reference DECODING FAILURES carry the entries that
meet 1e-5 in the reference's own fp32 and not in ours (tests/softparity.py FAILURE_BOUNDS).

For k = 1 .. 50 iterations, z (the final VC output, bp_vc.py:16-27) of every codeword from
  * ref64 / ref32 — the reference module itself in fp64 / fp32 (one reference layer looped, as make_golden.py),
  * ds     — the C oracle's (D, S) form (the GPU kernels' specification),
  * ops32  — the C oracle restating the reference's own fp32 operations (tanh, masked product, log((1+p)/(1-p))),
  * gpu    — the GPU decoder (optional: gpurun_out/trace_gpu.npz from scripts/trace_failure_gpu.py),
and after ONE iteration the check-to-variable messages (bp.py:46-47) of each, so the first operation where the
fp32 evaluations part is visible in isolation (iteration 1's VN input is the LLR alone).

Build container only (imports /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python scripts/trace_failure.py [--gpu gpurun_out/trace_gpu.npz] > profiles/r04/soft_trace.json
"""
import argparse
import json
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, "/root/reference/pytorch")
for p in ("ldpc-sims_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

np.complex = complex
np.float = float
from bp.bp import BeliefPropagation  # noqa: E402

import oracle  # noqa: E402
from ldpc_amd.codes import qc_expand  # noqa: E402
from softparity import decoded_rows  # noqa: E402

torch.set_num_threads(8)


def ref_per_iteration(H, llr, iters, clamp, double, chunk=32):
    """z after each iteration (iters, B, n) and the first iteration's c2v (B, E), the reference module itself."""
    model = BeliefPropagation(H, 1)
    model.eval()
    model = model.double() if double else model.float()
    dt = torch.float64 if double else torch.float32
    zs, x1s = [], []
    for s in range(0, llr.shape[0], chunk):
        L = torch.tensor(llr[s:s + chunk], dtype=dt)
        x = torch.zeros(L.shape[0], model.layer_size(), dtype=dt)
        per = []
        with torch.no_grad():
            for k in range(iters):
                x = model.layers[0]([x, -L]).clamp(-clamp, clamp)
                if k == 0:
                    x1s.append(x.numpy().copy())
                per.append(model.final_layer[0]([x, -L]).numpy().copy())
        zs.append(np.stack(per))
    return np.concatenate(zs, axis=1), np.concatenate(x1s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", default=os.path.join(ROOT, "gpurun_out", "trace_gpu.npz"))
    ap.add_argument("--tag", default="snr1")
    a = ap.parse_args()
    d = np.load(os.path.join(ROOT, "tests", "golden", "bp_wifi648_12_sp_it50.npz"))
    H = qc_expand(d["base"], int(d["Z"])).astype(np.int64)
    iters, clamp = int(d["iters"]), float(d["clamp"])
    llr = d[f"llr_{a.tag}"]
    z64, x64 = ref_per_iteration(H, llr, iters, clamp, True)
    z32, x32 = ref_per_iteration(H, llr, iters, clamp, False)
    assert np.array_equal(z64[-1], d[f"z_f64_{a.tag}"]) or np.abs(z64[-1] - d[f"z_f64_{a.tag}"]).max() < 1e-9
    assert np.array_equal(z32[-1].astype(np.float32), d[f"z_f32_{a.tag}"])
    ds = np.stack([oracle.sp_f32(H, llr, k, clamp, stable=True)["z"] for k in range(1, iters + 1)])
    ops = np.stack([oracle.sp_f32(H, llr, k, clamp)["z"] for k in range(1, iters + 1)])
    x1_ds = oracle.sp_f32(H, llr, 1, clamp, trace=True, stable=True)["trace"][0]
    x1_ops = oracle.sp_f32(H, llr, 1, clamp, trace=True)["trace"][0]
    gpu = np.load(a.gpu)["z"] if os.path.exists(a.gpu) else None   # (iters, B, n) from trace_failure_gpu.py
    conv = decoded_rows(H, z64[-1])

    def rel(z, k):
        return np.abs(z[k].astype(np.float64) - z64[k]) / np.maximum(1.0, np.abs(z64[k]))

    # the failing codeword with the most entries the reference's fp32 meets and ours (GPU, else the oracle) does not
    ours = gpu if gpu is not None else ds
    e_ours, e_ref = rel(ours, iters - 1), rel(z32, iters - 1)
    cnt = ((e_ours > 1e-5) & (e_ref <= 1e-5)).sum(axis=1) * ~conv
    c = int(np.argmax(cnt))
    out = {"golden": f"bp_wifi648_12_sp_it50.npz {a.tag}", "iters": iters, "clamp": clamp, "codeword": c,
           "decoded_codewords": int(conv.sum()), "codewords": int(conv.size),
           "entries_ref32_within_ours_not_at_50": {"ours": "gpu" if gpu is not None else "oracle-ds",
                                                   "this_codeword": int(cnt[c]), "all": int(cnt.sum())},
           "hard_bits_vs_codeword_at_k": [], "per_iteration": []}
    cw = d[f"codeword_{a.tag}"][c]
    for k in range(iters):
        row = {"k": k + 1}
        for name, z in (("gpu", gpu), ("ds", ds), ("ops32", ops), ("ref32", z32)):
            if z is not None:
                row[name] = float(rel(z, k)[c].max())
        row["bit_errors_ref64"] = int(((z64[k][c] < 0).astype(np.uint8) != cw).sum())
        row["gpu_vs_ref32"] = float((np.abs(ours[k][c].astype(np.float64) - z32[k][c]) /
                                     np.maximum(1.0, np.abs(z64[k][c]))).max())
        out["per_iteration"].append(row)
    first = {}
    for name in ("gpu", "ds", "ops32", "ref32"):
        ks = [r["k"] for r in out["per_iteration"] if r.get(name, 0.0) > 1e-5]
        first[name] = ks[0] if ks else None
    out["first_iteration_above_1e-5"] = first
    # iteration 1: c2v messages (check order) — the check-node output alone (the VN input is the LLR)
    sc = np.maximum(1.0, np.abs(x64[c]))
    out["iteration1_c2v_max_rel_vs_ref64"] = {
        "ds": float((np.abs(x1_ds[c] - x64[c]) / sc).max()), "ops32": float((np.abs(x1_ops[c] - x64[c]) / sc).max()),
        "ref32": float((np.abs(x32[c] - x64[c]) / sc).max())}
    out["growth_per_iteration"] = None
    err = [r.get("gpu", r["ds"]) for r in out["per_iteration"]]
    ks = [i for i in range(iters) if err[i] > 1e-7]
    if len(ks) > 5:
        k0, k1 = ks[0], iters - 1
        out["growth_per_iteration"] = float((err[k1] / err[k0]) ** (1.0 / max(1, k1 - k0)))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
