#!/usr/bin/env python3
"""Bitwise check of a library variant (LDPC_LIB=build_variants/X.so): the (1944,5/6) register kernel against the
generic CSR kernels, tanh-SP 50 iterations on 16-QAM OFDM LLRs (bits and z), odd B.  Exit status 1 on mismatch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ldpc-sims_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    import ldpc_amd
    from ldpc_amd.codes import get_code
    from test_gpu_config2 import _qam16_llrs
    H, _ = get_code("wifi1944_56")
    dec = ldpc_amd.get_decoder(H)
    _, x = _qam16_llrs(H, 1001, 6.0, seed=3)
    a = dec.decode(x, 50, algo="tanh", clamp=20.0, soft="z")
    b = dec.decode(x, 50, algo="tanh", clamp=20.0, soft="z", force_generic=True)
    ok = torch.equal(a["bits"], b["bits"]) and torch.equal(a["soft"].view(torch.int32), b["soft"].view(torch.int32))
    print(os.environ.get("LDPC_LIB", "default"), "bitwise equal to generic:", ok)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
