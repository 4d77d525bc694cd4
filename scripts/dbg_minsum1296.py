"""Debug: (1296,2/3) float min-sum register kernel vs oracle, current library (or LDPC_LIB)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ldpc-sims_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch
import ldpc_amd, oracle
from ldpc_amd.codes import get_code, Encoder
H, _ = get_code("wifi1296_23")
rng = np.random.default_rng(11)
enc = Encoder(H)
cw = enc.encode(rng.integers(0, 2, size=(1000, enc.k)))
rate = enc.k / H.shape[1]
sigma = np.sqrt(1.0 / (2 * rate * 10 ** (4.0 / 10)))
llr = (-2.0 * ((1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)) / sigma**2).astype(np.float32)
llr[0] = 0.0; llr[1, ::3] = 0.0; llr[2] = np.float32(1e30)
dec = ldpc_amd.get_decoder(H)
for algo, kw in (("minsum", {}), ("tanh", {}), ("qminsum", {})):
    for es in (False, True):
        r = dec.decode(torch.from_numpy(llr).cuda(), 25, algo=algo, clamp=20.0, soft="z", early_stop=es, want_iters=True, **kw)
        if algo == "minsum":
            ref = oracle.ms_f32(H, llr, 25, 20.0, early_stop=es)
            zr = ref["z"]
        elif algo == "tanh":
            ref = oracle.sp_f32(H, llr, 25, 20.0, early_stop=es, stable=True); zr = ref["z"]
        else:
            q = np.clip(np.rint(llr), -15, 15).astype(np.int8)
            ref = oracle.qms(H, q, 25, 15, 127, 0, early_stop=es); zr = (0.5 * ref["app"]).astype(np.float32)
        b = r["bits"].cpu().numpy(); z = r["soft"].cpu().numpy()
        rows = np.nonzero((b != ref["bits"]).any(1))[0]
        zd = np.nonzero((np.abs(z - zr) > 1e-4 * np.maximum(1, np.abs(zr))).any(1))[0]
        it = (r["iters_used"].cpu().numpy() != ref["iters_used"]).sum()
        print(os.environ.get("LDPC_LIB", "current"), algo, "es" if es else "fixed", "bit rows", rows[:12].tolist(), len(rows),
              "z rows", zd[:12].tolist(), len(zd), "iters mismatches", int(it), flush=True)
