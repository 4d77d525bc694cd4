"""GPU, maximum sizes: batches whose element index passes 2^31, so every kernel's codeword offsets must be
64-bit (the QC register kernels, the sliced Z = 81 kernels and the generic CSR kernels with their
workspace of ~70 GB).  Rows at the head, around the 2^31-element boundary and at the tail are checked
against the oracle (min-sum: bit for bit, soft z included) or against the generic kernels (tanh-SP: the
QC kernel equals them bitwise), decoded there as a small batch."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd.codes import get_code  # noqa: E402


def _rows(B, n):
    r0 = (1 << 31) // n
    return np.unique(np.r_[0:32, r0 - 32:r0 + 32, B - 32:B])


@pytest.mark.parametrize("code,algo,force_generic", [
    ("wifi648_12", "minsum", False), ("wifi648_12", "minsum", True), ("wifi648_12", "tanh", False),
    ("wifi1944_56", "minsum", False)])
def test_batch_beyond_2g_elements(code, algo, force_generic):
    H, _ = get_code(code)
    n = H.shape[1]
    B = (1 << 31) // n + 2048                      # B * n > 2^31
    g = torch.Generator(device="cuda").manual_seed(7)
    llr = torch.randn((B, n), device="cuda", generator=g) * 3.0 + 1.0
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(llr, 8, algo=algo, clamp=20.0, soft="z", force_generic=force_generic)
    torch.cuda.synchronize()
    rows = torch.from_numpy(_rows(B, n)).cuda()
    x = llr[rows].cpu().numpy()
    bits, z = r["bits"][rows].cpu().numpy(), r["soft"][rows].cpu().numpy()
    del r, llr
    torch.cuda.empty_cache()
    if algo == "minsum":
        ref = oracle.ms_f32(H, x, 8, 20.0)
        assert np.array_equal(bits, ref["bits"])
        assert np.array_equal(z.view(np.uint32), ref["z"].view(np.uint32))
    else:
        ref = dec.decode(torch.from_numpy(x).cuda(), 8, algo=algo, clamp=20.0, soft="z", force_generic=True)
        assert np.array_equal(bits, ref["bits"].cpu().numpy())
        assert np.array_equal(z.view(np.uint32), ref["soft"].cpu().numpy().view(np.uint32))
