"""Decode fixed seeded inputs with the library named by LDPC_LIB and save every output (bits, soft z,
iters) to an npz; `--compare a.npz b.npz` checks two such files bit for bit.  Used to show that a kernel
rewrite leaves results unchanged (e.g. restated division/logf, scheduling variants).

  LDPC_LIB=build_variants/base.so python scripts/cmp_libs.py out_a.npz
  python scripts/cmp_libs.py out_b.npz && python scripts/cmp_libs.py --compare out_a.npz out_b.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ldpc-sims_amd"))


def cases():
    # (code, algo, iters, kw); inputs: AWGN LLRs at a waterfall SNR plus saturating and zero entries
    for code in ("peg64_32", "wifi648_12", "wifi1296_23", "wifi1944_56"):
        for algo in ("tanh", "minsum", "qminsum"):
            for fg in (False, True):
                yield code, algo, 12, dict(force_generic=fg)
        yield code, "minsum", 20, dict(early_stop=True)
        yield code, "tanh", 12, dict(precision="f64", force_generic=True)


def run(out):
    import torch
    import ldpc_amd
    from ldpc_amd import codes
    res = {}
    for i, (code, algo, iters, kw) in enumerate(cases()):
        H, _ = codes.get_code(code)
        n = H.shape[1]
        rng = np.random.default_rng(100 + i)
        B = 1000
        llr = (rng.standard_normal((B, n)) * 3.0 + 1.5).astype(np.float32)
        llr[0, :7] = 1e4
        llr[1, :5] = 0.0
        if kw.get("precision") == "f64":
            llr = llr.astype(np.float64)
        dec = ldpc_amd.get_decoder(H)
        try:
            r = dec.decode(llr, iters, algo=algo, clamp=10.0, soft="z", want_iters=True, **kw)
        except Exception as e:  # unsupported combination: recorded as such on both sides
            print("skip", code, algo, kw, e)
            continue
        key = f"{i}_{code}_{algo}_{'_'.join(f'{k}{v}' for k, v in kw.items())}"
        res[key + "_bits"] = r["bits"]
        res[key + "_z"] = r["soft"].view(np.uint64 if r["soft"].dtype == np.float64 else np.uint32)
        if r.get("iters_used") is not None:
            res[key + "_it"] = r["iters_used"]
    np.savez(out, **res)
    print("wrote", out, len(res))


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k], Bz[k])]
    print(f"{len(A.files) - len(bad)}/{len(A.files)} arrays identical")
    for k in bad:
        print("DIFF", k, int((A[k] != Bz[k]).sum()))
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])
