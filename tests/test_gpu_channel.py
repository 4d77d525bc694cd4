"""OFDM front end on device vs the reference's demodulate_signal (golden) and numpy restatements."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from softparity import _log

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
from ldpc_amd.channel import ofdm_demod, ofdm_tx  # noqa: E402


def _np_map(bits, bps):
    b = bits.reshape(-1, bps).astype(np.float64)
    if bps == 2:
        return ((1 - 2 * b[:, 0]) + 1j * (1 - 2 * b[:, 1])) / np.sqrt(2)
    return ((1 - 2 * b[:, 0]) * (3 - 2 * b[:, 1]) + 1j * (1 - 2 * b[:, 2]) * (3 - 2 * b[:, 3])) / np.sqrt(10)


def _dft(N):
    x = np.arange(N)
    return np.exp(-2j * np.pi * np.outer(x, x) / N) / np.sqrt(N)


def test_demod_matches_reference_golden():
    d = np.load(os.path.join(GOLDEN, "demod_ofdm.npz"))     # ofdm_functions.demodulate_signal output
    rx = torch.from_numpy(d["rx"].astype(np.complex64)).cuda()
    snr = 10 ** (float(d["snr_db"]) / 10)
    llr, sym = ofdm_demod(rx, int(d["ofdm_size"]), 2, snr, want_symbols=True)
    ref = d["llrs"].reshape(-1)
    got = llr.cpu().numpy().astype(np.float64)
    rel = float((np.abs(got - ref) / np.maximum(1.0, np.abs(ref))).max())
    _log({"label": "demod_ofdm qpsk", "kind": "llr_rel_vs_reference", "max": rel})
    assert rel <= 5e-6   # measured 7.1e-7 (profiles/r02/soft_parity.jsonl): fp32 DFT vs the reference's fp64
    assert np.allclose(sym.cpu().numpy(), d["rx_symbols"].reshape(-1), atol=1e-5)


@pytest.mark.parametrize("bps", [2, 4])
def test_tx_is_unitary_idft_and_roundtrips(bps):
    rng = np.random.default_rng(bps)
    N, nsym = 32, 32 * 40
    bits = rng.integers(0, 2, size=nsym * bps).astype(np.uint8)
    rx, tx = ofdm_tx(torch.from_numpy(bits).cuda(), N, bps, snr=1e12, seed=1, want_tx=True)
    s = _np_map(bits, bps).reshape(-1, N).T                # columns = OFDM blocks (transmit_symbols:26)
    want = (_dft(N).conj().T @ s).T.reshape(-1)
    assert np.abs(tx.cpu().numpy() - want).max() < 2e-6
    llr, sym = ofdm_demod(rx, N, bps, snr=1e3, want_symbols=True)
    assert np.abs(sym.cpu().numpy() - _np_map(bits, bps)).max() < 2e-5
    assert np.array_equal((llr.cpu().numpy() > 0).astype(np.uint8), bits)


def test_16qam_llr_is_exact_logsumexp():
    rng = np.random.default_rng(3)
    N, nsym, snr = 32, 32 * 64, 4.0
    bits = rng.integers(0, 2, size=nsym * 4).astype(np.uint8)
    rx = ofdm_tx(torch.from_numpy(bits).cuda(), N, 4, snr=snr, seed=5)
    llr, sym = ofdm_demod(rx, N, 4, snr, want_symbols=True)
    y = sym.cpu().numpy().astype(np.complex128)
    np_ = 0.5 / snr
    lv = np.array([3, 1, -1, -3]) / np.sqrt(10)                 # (ba,bb) = 00, 01, 11, 10
    ba = np.array([0, 0, 1, 1])
    bb = np.array([0, 1, 1, 0])

    def dim(v):
        m = -(v[:, None] - lv[None, :]) ** 2 / (2 * np_)
        lse = lambda mm, sel: np.logaddexp.reduce(np.where(sel[None, :], mm, -np.inf), axis=1)
        return lse(m, ba == 1) - lse(m, ba == 0), lse(m, bb == 1) - lse(m, bb == 0)

    la, lb = dim(y.real)
    lc, ld = dim(y.imag)
    want = np.stack([la, lb, lc, ld], axis=1).reshape(-1)
    got = llr.cpu().numpy()
    assert np.allclose(got, want, rtol=1e-4, atol=1e-3)


def test_qpsk_ofdm_llr_statistics_equal_bpsk_equivalent():
    """All-zero bits: LLR ~ N(-2 snr, 4 snr) — the distribution the BPSK/AWGN shortcut uses."""
    N, nsym, snr = 32, 32 * 8192, 2.0
    bits = torch.zeros(nsym * 2, dtype=torch.uint8, device="cuda")
    llr = ofdm_demod(ofdm_tx(bits, N, 2, snr, seed=9), N, 2, snr).double()
    assert abs(llr.mean().item() + 2 * snr) < 0.02 * 2 * snr
    assert abs(llr.var().item() - 4 * snr) < 0.02 * 4 * snr


A = np.load(os.path.join(GOLDEN, "adc_quantizer.npz"))


def test_adc_fixed_clip_matches_reference():
    from ldpc_amd.channel import adc_quantize
    rx = torch.from_numpy(A["rx"].astype(np.complex64)).cuda()
    for i, (b, c) in enumerate(A["fixed"]):
        q = adc_quantize(rx, int(b), clip_value=float(c)).cpu().numpy()
        assert np.array_equal(q, A[f"q_fixed{i}"].astype(np.complex64)), (b, c)


def test_gen_qdata_agc_matches_reference():
    from ldpc_amd.channel import adc_quantize, gen_qdata
    rx = torch.from_numpy(A["rx"].astype(np.complex64)).cuda()
    for i, (b, r) in enumerate(A["agc"]):
        _, clip = adc_quantize(rx, int(b), clip_ratio=float(r), want_clip=True)
        assert np.isclose(clip.item(), float(A[f"clip_agc{i}"]), rtol=1e-12)
        q, qs, ql = gen_qdata(rx, float(A["snr_db"]), int(b), float(r), int(A["ofdm_size"]))
        assert np.array_equal(q.cpu().numpy(), A[f"q_agc{i}"].astype(np.complex64)), (b, r)
        assert np.abs(qs.cpu().numpy() - A[f"qsym_agc{i}"]).max() < 1e-5
        ref = A[f"qllr_agc{i}"]
        assert np.allclose(ql.cpu().numpy(), ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())
