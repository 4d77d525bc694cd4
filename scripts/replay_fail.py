"""Replay a parity-sweep failing batch (scripts/parity_stress.py's stress_fail_<n>.npz) through the library in use
(LDPC_LIB picks a variant build) and report, for the tanh-SP codewords that converge at the recorded iteration, the
z distance of the GPU, of the oracle's (D, S) fp32 form and of the reference's fp32 module from the reference's fp64
arithmetic, and the GPU's distance from the oracle.
    python scripts/replay_fail.py gpurun_out/stress/stress_fail_1.npz ..."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ldpc-sims_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import ldpc_amd  # noqa: E402
import oracle  # noqa: E402
from ldpc_amd.codes import get_code  # noqa: E402

for f in sys.argv[1:]:
    d = np.load(f)
    x, desc = d["llr"], json.loads(str(d["desc"]))
    H, _ = get_code(desc["code"])
    iters, clamp, es = desc["iters"], desc["clamp"], desc["early_stop"]
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(torch.from_numpy(x).cuda(), iters, algo="tanh", clamp=clamp, early_stop=es, soft="z",
                   want_iters=True)
    torch.cuda.synchronize()
    gz, gu = r["soft"].cpu().numpy(), r["iters_used"].cpu().numpy()
    ref = oracle.sp_f32(H, x, iters, clamp, early_stop=es, stable=True)
    target = desc["spec"]["converged_at"]
    print(f"{os.path.basename(f)} {desc['code']} path {dec.kernel_path(dec.params(iters, 'tanh', clamp))} "
          f"lib {os.environ.get('LDPC_LIB', 'in-tree')}")
    for c in np.nonzero(ref["iters_used"] == target)[0]:
        it = int(gu[c]) if es else iters
        o64 = oracle.sp_f64(H, x[c:c + 1].astype(np.float64), it, clamp, ceiling="f32")["z"][0]
        rz = oracle.sp_f32(H, x[c:c + 1], it, clamp, stable=False)["z"][0]
        sc = np.maximum(np.abs(o64), 1.0)
        e = lambda z: float((np.abs(z - o64) / sc).max())  # noqa: E731
        print(f"  cw {c:4d} it {it:2d}  gpu {e(gz[c]):.3g}  oracle {e(ref['z'][c]):.3g}  ref32 {e(rz):.3g}  "
              f"gpu-vs-oracle {float((np.abs(gz[c] - ref['z'][c]) / np.maximum(np.abs(ref['z'][c]), 1.0)).max()):.3g}"
              f"  bitwise-equal-to-oracle {bool(np.array_equal(gz[c].view(np.int32), ref['z'][c].view(np.int32)))}")
