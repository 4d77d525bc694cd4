#!/usr/bin/env python3
"""GPU half of the config [2] reference golden (tests/golden/make_golden.py part `wifi1944c2`): 16 codewords of
the (1944,5/6) code per Eb/N0 point through the on-device 16-QAM OFDM front end exactly as bench.py's config [2]
leg and tests/test_gpu_config2.py generate them (random info bits, systematic encoder, ofdm_tx / ofdm_demod with
ofdm_size 32).  Writes gpurun_out/c2_16qam_llrs.npz (codewords uint8, LLRs float32, log P1/P0), which is copied
to tests/golden/c2_16qam_llrs.npz and fed to the reference in the build container.

    python scripts/gen_c2_llrs_gpu.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ldpc-sims_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    from ldpc_amd.codes import get_code
    from test_gpu_config2 import _qam16_llrs
    H, _ = get_code("wifi1944_56")
    rec = {}
    for ebn0 in (6.0, 6.5):
        cw, x = _qam16_llrs(H, 16, ebn0, seed=700 + int(ebn0 * 10))
        tag = f"snr{ebn0:g}".replace(".", "p")
        rec[f"codeword_{tag}"] = cw.astype(np.uint8)
        rec[f"llr_{tag}"] = x.cpu().numpy().astype(np.float32)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "c2_16qam_llrs.npz"), snrs=np.array([6.0, 6.5]), **rec)
    print("c2_16qam_llrs.npz", {k: v.shape for k, v in rec.items()})


if __name__ == "__main__":
    main()
