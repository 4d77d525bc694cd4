"""BASELINE config [2] at its own iteration count: 802.11n (1944,5/6) tanh sum-product, 50 iterations, on 16-QAM
OFDM LLRs from the on-device front end — exactly the leg bench.py times (side.configs.config2) — against the C
oracle's (D, S)-form fp32 restatement (oracle.sp_f32(stable=True), the kernels' specification; restating
bp_vc.py:16-27 / bp_cv.py:22-50), on 256 codewords per point.  The REFERENCE's own run of this configuration (32
codewords of the same front end, one reference layer looped: tests/golden/bp_wifi1944_56_sp_it50_cl20.npz — bits,
p1 and z against its fp32 module and the f32-bound .double()) is checked by tests/test_gpu_soft_parity.py with
every other golden.

Tolerances (the soft target is the fp64 evaluation of the same function, oracle.sp_f64 with the fp32 module's
p-clamp bound since clamp 20 is above the ceiling — pinned to the reference's own fp64 module in
test_oracle_golden.py): hard bits identical to the oracle on every codeword it decodes (zero syndrome, and
they are the transmitted codewords); z within 1e-5 relative (scale max(1, |z|)) of the fp64 target on every
codeword that converged at least 10 iterations before the end (the oracle's early-stop iteration count); on the
codewords that converged in the last 10 iterations, the fp32 trajectory was chaotic until then — the oracle's
own fp32 is 1.3e-5 .. 6.3e-5 from fp64 there (measured) — so z within 1e-4 (measured 3.8e-5 with the fma join,
7.4e-5 before it); on
decoding failures only the count is compared."""
import numpy as np
import pytest

import oracle
from softparity import _log

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd.channel import ofdm_demod, ofdm_tx  # noqa: E402
from ldpc_amd.codes import Encoder, get_code  # noqa: E402

TOL_Z_REL = 1e-5
TOL_Z_REL_LATE = 1e-4


def _qam16_llrs(H, B, ebn0, seed):
    """(codewords, LLRs) of B random codewords through 16-QAM OFDM (ofdm_size 32) at Eb/N0, as bench.py does."""
    n = H.shape[1]
    rate = 1 - H.shape[0] / n
    enc = Encoder(H)
    rng = np.random.default_rng(seed)
    cw = enc.encode(rng.integers(0, 2, size=(B, enc.k))).astype(np.uint8)
    s = torch.from_numpy(cw.reshape(-1)).cuda()
    pad = (-s.numel()) % (4 * 32)
    if pad:
        s = torch.cat([s, torch.zeros(pad, dtype=torch.uint8, device="cuda")])
    esn0 = float(10.0 ** (ebn0 / 10.0) * rate * 4)
    rx = ofdm_tx(s, 32, 4, esn0, seed, 0)
    llr = ofdm_demod(rx, 32, 4, esn0)[:B * n].view(B, n).contiguous()
    return cw, llr


@pytest.mark.parametrize("ebn0", [6.0, 6.5])
def test_config2_tanh50_16qam_vs_oracle(ebn0):
    H, _ = get_code("wifi1944_56")
    B = 256
    cw, x = _qam16_llrs(H, B, ebn0, seed=40 + int(ebn0 * 10))
    dec = ldpc_amd.get_decoder(H)
    assert dec.qc_z == 81
    r = dec.decode(x, 50, algo="tanh", clamp=20.0, soft="z")    # bench's config [2] leg: clamp 20, 50 it
    llr = x.cpu().numpy()
    ref = oracle.sp_f32(H, llr, 50, 20.0, stable=True)
    conv_at = oracle.sp_f32(H, llr, 50, 20.0, stable=True, early_stop=True)["iters_used"]
    t64 = oracle.sp_f64(H, llr.astype(np.float64), 50, 20.0, ceiling="f32")["z"]
    g = ldpc_amd.codes.Graph.from_H(H)
    par = np.add.reduceat(ref["bits"][:, g.col_idx].astype(np.int64), g.row_ptr[:-1], axis=1) % 2
    ok = ~par.any(axis=1)
    bits = r["bits"].cpu().numpy()
    gpar = np.add.reduceat(bits[:, g.col_idx].astype(np.int64), g.row_ptr[:-1], axis=1) % 2
    assert ok.sum() >= B // 4, ok.sum()                      # enough decoded codewords to mean something
    assert np.array_equal(bits[ok], ref["bits"][ok])
    assert np.array_equal(ref["bits"][ok], cw[ok])           # and they are the transmitted codewords
    assert abs(int((~gpar.any(axis=1)).sum()) - int(ok.sum())) <= max(1, B // 32)
    z = r["soft"].cpu().numpy().astype(np.float64)
    rel = np.abs(z - t64) / np.maximum(1.0, np.abs(t64))
    early = ok & (conv_at <= 40)
    late = ok & (conv_at > 40)
    rec = {"label": f"config2 wifi1944_56 tanh 50 it 16-QAM {ebn0} dB", "kind": "z_rel_vs_f64",
           "decoded": int(ok.sum()), "of": B, "converged_by_40": int(early.sum()),
           "max_converged_by_40": float(rel[early].max()), "tol": TOL_Z_REL,
           "converged_after_40": int(late.sum()), "max_converged_after_40": float(rel[late].max()) if late.any() else 0.0,
           "tol_late": TOL_Z_REL_LATE}
    _log(rec)
    assert early.sum() >= B // 4 and rel[early].max() <= TOL_Z_REL, rec
    assert rec["max_converged_after_40"] <= TOL_Z_REL_LATE, rec


def test_config2_kernels_agree_at_50_iterations():
    """The on-chip sliced kernel and the generic CSR kernels perform the same operations in the same order:
    bits and z bitwise equal at config [2]'s 50 iterations on its 16-QAM LLRs (decoded and failing codewords
    alike), including a ragged batch (odd B: the last unit's second codeword is absent)."""
    H, _ = get_code("wifi1944_56")
    dec = ldpc_amd.get_decoder(H)
    for B, e in ((301, 6.0), (64, 5.5)):
        _, x = _qam16_llrs(H, B, e, seed=7 + B)
        a = dec.decode(x, 50, algo="tanh", clamp=20.0, soft="z")
        b = dec.decode(x, 50, algo="tanh", clamp=20.0, soft="z", force_generic=True)
        assert torch.equal(a["bits"], b["bits"])
        assert torch.equal(a["soft"].view(torch.int32), b["soft"].view(torch.int32))


@pytest.mark.parametrize("B", [1, 2, 3])
def test_config2_resident_kernel_tiny_batches_write_nothing_past_B(B):
    """The resident kernel decodes codeword pairs (one unit = two codewords in the lane halves): B = 1 and 3
    leave the last unit's second codeword absent.  Bits and z bitwise equal to the generic CSR path, and the
    rows after B of larger output buffers stay untouched."""
    from ldpc_amd import _abi
    H, _ = get_code("wifi1944_56")
    n = H.shape[1]
    dec = ldpc_amd.get_decoder(H)
    _, x = _qam16_llrs(H, B, 6.0, seed=90 + B)
    a = dec.decode(x, 50, algo="tanh", clamp=20.0, soft="z")
    g = dec.decode(x, 50, algo="tanh", clamp=20.0, soft="z", force_generic=True)
    assert torch.equal(a["bits"], g["bits"]) and torch.equal(a["soft"].view(torch.int32), g["soft"].view(torch.int32))
    p = dec.params(50, "tanh", 20.0, 1.0, 0.0, False, "f32", "z", device_ptrs=True)
    bits = torch.full((B + 2, n), 7, dtype=torch.uint8, device="cuda")
    soft = torch.full((B + 2, n), 7.0, dtype=torch.float32, device="cuda")
    used = torch.full((B + 2,), 77, dtype=torch.int32, device="cuda")
    ws = torch.empty((max(dec.workspace_bytes(B, p), 1),), dtype=torch.uint8, device="cuda")
    _abi.check(dec.lib.ldpc_decode_ex(dec._h, x.data_ptr(), B, p, bits.data_ptr(), soft.data_ptr(), used.data_ptr(),
                                      ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert (bits[B:] == 7).all() and (soft[B:] == 7.0).all() and (used[B:] == 77).all()
    assert torch.equal(bits[:B], a["bits"]) and (used[:B] == 50).all()
