"""Statistical pin: the reference's only published numbers — the (64,32) BER/BLER curve in
pytorch/outputs/ber/20191203-191640_tx=20191203-162534_quantized.pkl (tanh-SP, 3 iterations, clamp 20,
65,536 codewords per point; written by evaluate_quantized.py:153-175; values transcribed in BASELINE.md
and SURVEY.md §6) — reproduced by the GPU decoder through the sweep driver."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from ldpc_amd.sweep import run  # noqa: E402

SNR = list(range(11))
PUB_UNCODED = [0.15891, 0.13101, 0.10402, 0.07875, 0.05647, 0.03750, 0.02295, 0.01258, 0.00595, 0.00240, 0.00077]
PUB_BER = [7.271e-2, 4.467e-2, 2.450e-2, 1.142e-2, 4.457e-3, 1.411e-3, 3.419e-4, 6.151e-5, 8.106e-6, 9.537e-7, 0.0]
PUB_BLER = [8.776e-1, 7.269e-1, 5.136e-1, 2.926e-1, 1.276e-1, 4.373e-2, 1.086e-2, 1.953e-3, 2.747e-4, 3.052e-5, 0.0]
N = 65536


def test_reproduces_published_curve():
    r = run("peg64_32", "tanh", 3, 20.0, snr_db=SNR, codewords=N, batch=N, seed=11)
    assert r["codewords"].tolist() == [N] * 11
    for i in SNR:
        # two independent estimates with N codewords each: sigma of the difference, 5 sigma + 2 counts
        pb = max(PUB_BLER[i], 1.0 / N)
        tol_bler = 5 * np.sqrt(2 * pb * (1 - pb) / N) + 2.0 / N
        pe = max(PUB_BER[i], 1.0 / (32 * N))
        tol_ber = 5 * np.sqrt(2 * pe / N) + 2.0 / (32 * N)          # bits within a codeword correlated
        pu = PUB_UNCODED[i]
        tol_unc = 5 * np.sqrt(2 * pu * (1 - pu) / (64 * N))
        assert abs(r["coded_bler"][i] - PUB_BLER[i]) <= tol_bler, (i, r["coded_bler"][i], PUB_BLER[i])
        assert abs(r["coded_ber"][i] - PUB_BER[i]) <= tol_ber, (i, r["coded_ber"][i], PUB_BER[i])
        assert abs(r["uncoded_ber"][i] - PUB_UNCODED[i]) <= tol_unc, (i, r["uncoded_ber"][i], PUB_UNCODED[i])


def test_sweep_shard_independent_data():
    """Codeword content and noise are keyed by the global codeword index: one 4096-codeword shard of a
    sweep equals the same rows of the unsharded run (what makes multi-GPU sweeps reproducible)."""
    a = run("wifi648_12", "minsum", 10, 20.0, snr_db=[2.0], codewords=8192, batch=8192, seed=3)
    b0 = run("wifi648_12", "minsum", 10, 20.0, snr_db=[2.0], codewords=8192, batch=8192, seed=3, rank=0, world=2)
    b1 = run("wifi648_12", "minsum", 10, 20.0, snr_db=[2.0], codewords=8192, batch=8192, seed=3, rank=1, world=2)
    # without a process group each rank keeps its own counts: they must add up to the unsharded run
    tot = b0["coded_bler"] * b0["codewords"] + b1["coded_bler"] * b1["codewords"]
    assert np.allclose(tot, a["coded_bler"] * a["codewords"])
