"""Exact-zero LLRs (erasures) through the register QC min-sum kernels at 0, 1 and 2 iterations: z bit for bit
against the oracle, signs of zero included.  The oracle forms APP_0 = -llr + sum of the initial c2v (+0), so an
erased variable starts at +0, and iteration 0's v2c = APP_0 - c2v is +0 too; the kernels used to start from -llr
itself (-0) — invisible in the bits and in p1, visible in z.  Found by scripts/parity_stress.py (round 5)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd.codes import Encoder, get_code  # noqa: E402


@pytest.mark.parametrize("name", ["wifi648_12", "wifi1296_23", "wifi1944_56"])
@pytest.mark.parametrize("early_stop", [False, True])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (0.8125, 0.5)])
def test_erasures_few_iterations_bitwise(name, early_stop, alpha, beta):
    H, _ = get_code(name)
    dec = ldpc_amd.get_decoder(H)
    rng = np.random.default_rng(3)
    enc = Encoder(H)
    B = 67
    cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
    x = (-2.0 * ((1.0 - 2.0 * cw) + 0.8 * rng.standard_normal(cw.shape)) / 0.64).astype(np.float32)
    x[rng.random(x.shape) < 0.08] = 0.0
    x[0, :] = 0.0                                            # an all-erased codeword
    x[1, ::2] = -0.0                                         # negative zeros
    xg = torch.from_numpy(x).cuda()
    for iters in (0, 1, 2):
        assert dec.kernel_path(dec.params(iters, "minsum", 20.0, alpha=alpha, beta=beta,
                                          early_stop=early_stop)).startswith("qc-")
        r = dec.decode(xg, iters, algo="minsum", clamp=20.0, alpha=alpha, beta=beta, early_stop=early_stop,
                       soft="z", want_iters=True)
        torch.cuda.synchronize()
        ref = oracle.ms_f32(H, x, iters, 20.0, alpha, beta, early_stop=early_stop)
        z = r["soft"].cpu().numpy()
        assert np.array_equal(r["bits"].cpu().numpy(), ref["bits"]), iters
        assert np.array_equal(r["iters_used"].cpu().numpy(), ref["iters_used"]), iters
        bad = z.view(np.uint32) != ref["z"].view(np.uint32)
        assert not bad.any(), (iters, int(bad.sum()), z[bad][:4], ref["z"][bad][:4])
