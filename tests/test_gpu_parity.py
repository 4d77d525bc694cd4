"""GPU parity: the HIP decoder (through libldpc_hip.so's C ABI) against the reference's golden vectors and
the CPU oracle.  Tolerances are stated per test; hard decisions must match exactly."""
import glob
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from softparity import _log, check_p1

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd import _abi  # noqa: E402
from ldpc_amd.codes import Encoder, get_code  # noqa: E402

PEG_FILES = sorted(glob.glob(os.path.join(GOLDEN, "bp_peg64_snr*.npz")))
# fp32 soft outputs: 1e-5 against the reference's fp64 p1 on its well-conditioned entries
# (tests/softparity.py); fp64: against the reference's .double() module.
TOL_P1_F64_VS_REF = 1e-10
# GPU fp32 z against the C oracle's (D, S)-form fp32 z at 8 iterations: the same operations with the device
# library's exp/log/rcp instead of glibc's expf/logf and a correctly rounded division — ulp-level differences,
# no cancellation to amplify them.  The round-2 tanh/log form needed 1e-4 here (measured 4.4e-5).
TOL_Z_REL_VS_ORACLE = 1e-5


def _llr(H, B, snr_db, seed, rate=0.5):
    rng = np.random.default_rng(seed)
    enc = Encoder(H)
    cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
    sigma = np.sqrt(1.0 / (2 * rate * 10 ** (snr_db / 10)))
    y = (1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)
    return cw, (-2.0 * y / sigma**2).astype(np.float32)


@pytest.fixture(scope="module", params=[False, True], ids=["auto", "generic"])
def force_generic(request):
    return request.param


@pytest.mark.parametrize("path", PEG_FILES, ids=lambda p: os.path.basename(p))
def test_sp_f32_matches_reference_golden(path):
    d = np.load(path)
    dec = ldpc_amd.get_decoder(d["H"])
    r = dec.decode(torch.from_numpy(d["llr"]).cuda(), int(d["iters"]), algo="tanh", clamp=float(d["clamp"]), soft="p1")
    assert np.array_equal(r["bits"].cpu().numpy(), d["bits_f32"])
    check_p1("peg64 " + os.path.basename(path)[:-4], r["soft"].cpu().numpy(), d["p1_f32"], d["p1_f64"], d["H"])


@pytest.mark.parametrize("path", PEG_FILES, ids=lambda p: os.path.basename(p))
def test_sp_f64_matches_reference_golden(path):
    d = np.load(path)
    dec = ldpc_amd.get_decoder(d["H"])
    r = dec.decode(d["llr"].astype(np.float64), int(d["iters"]), algo="tanh", clamp=float(d["clamp"]),
                   precision="f64", soft="p1")
    assert np.array_equal(r["bits"], d["bits_f64"])
    assert np.abs(r["soft"] - d["p1_f64"]).max() <= TOL_P1_F64_VS_REF


def test_decode_bits_dropin_matches_reference_golden():
    d = np.load(os.path.join(GOLDEN, "decode_bits_peg64.npz"))
    out = ldpc_amd.decode_bits(d["llrs"], d["H"], int(d["iters"]), int(d["batch_size"]), int(d["clamp"]))
    assert out.dtype == np.float64 and out.shape == d["out"].shape
    assert np.array_equal(out, d["out"])
    with pytest.raises(ZeroDivisionError):
        ldpc_amd.decode_bits(d["llrs"], d["H"], 5, 0, 10)
    # the recycled-buffer result vs the opt-out: same values, a fresh self-owning array
    fresh = ldpc_amd.decode_bits(d["llrs"], d["H"], int(d["iters"]), int(d["batch_size"]), int(d["clamp"]),
                                 fresh_output=True)
    assert fresh.flags.owndata and not out.flags.owndata
    assert np.array_equal(fresh, d["out"]) and fresh.dtype == np.float64
    fresh.resize((fresh.shape[0] * fresh.shape[1],), refcheck=False)   # a plain numpy array: resizable


@pytest.mark.parametrize("chunk", [7, 48, 1000])
def test_decode_bits_host_pipeline_chunks(chunk):
    """ldpc_decode_bits_host (the pipelined drop-in) with chunks smaller than, equal to and larger than the
    decoded rows: 96 of the golden's 100 rows in 14 / 2 / 1 chunks (ragged last chunk), bit-identical to
    the reference's decode_bits output; rows past `rows` untouched; invalid flags rejected."""
    import ctypes
    d = np.load(os.path.join(GOLDEN, "decode_bits_peg64.npz"))
    dec = ldpc_amd.get_decoder(d["H"])
    p = dec.params(int(d["iters"]), "tanh", float(d["clamp"]))
    x = np.ascontiguousarray(d["llrs"], np.float64)
    out = np.full(x.shape, 7.0)
    _abi.check(dec.lib.ldpc_decode_bits_host(dec._h, x.ctypes.data, 96, ctypes.byref(p), out.ctypes.data, chunk, 3))
    assert np.array_equal(out[:96], d["out"][:96])
    assert (out[96:] == 7.0).all()
    for bad in (_abi.F_F64, _abi.F_DEVICE_PTRS, _abi.F_SOFT_Z):
        q = dec.params(5, "tanh", 10.0)
        q.flags |= bad
        assert dec.lib.ldpc_decode_bits_host(dec._h, x.ctypes.data, 96, ctypes.byref(q), out.ctypes.data, 0, 0) \
            == _abi.LDPC_EINVAL


def test_ldpc_decode_short_form_with_iters_used():
    """ldpc_decode (the SURVEY §8(b) signature, host pointers, internal workspace) against the reference's
    golden bits and against ldpc_decode_ex: same bits, p1 bitwise, and iters_used filled — the fixed count
    without early stop, the per-codeword counts of ldpc_decode_ex with LDPC_F_EARLY_STOP."""
    import ctypes
    d = np.load(os.path.join(GOLDEN, "decode_bits_peg64.npz"))
    H = d["H"]
    dec = ldpc_amd.get_decoder(H)
    x = np.ascontiguousarray(d["llrs"], np.float32)
    B, n = x.shape
    it, cl = int(d["iters"]), float(d["clamp"])
    for flags in (0, _abi.F_EARLY_STOP):
        bits = np.empty((B, n), np.uint8)
        p1 = np.empty((B, n), np.float32)
        used = np.full(B, -1, np.int32)
        _abi.check(dec.lib.ldpc_decode(dec._h, x.ctypes.data, B, it, cl, _abi.ALGO_TANH_SP, flags, bits.ctypes.data,
                                       p1.ctypes.data, used.ctypes.data, None))
        p = dec.params(it, "tanh", cl, early_stop=bool(flags))
        bits2 = np.empty_like(bits)
        p12 = np.empty_like(p1)
        used2 = np.full(B, -2, np.int32)
        _abi.check(dec.lib.ldpc_decode_ex(dec._h, x.ctypes.data, B, ctypes.byref(p), bits2.ctypes.data,
                                          p12.ctypes.data, used2.ctypes.data, None, 0, None))
        assert np.array_equal(bits, bits2) and np.array_equal(p1.view(np.uint32), p12.view(np.uint32))
        assert np.array_equal(used, used2)
        if flags == 0:
            assert (used == it).all()
            rows = (B // int(d["batch_size"])) * int(d["batch_size"])
            assert np.array_equal(bits[:rows].astype(np.float64), d["out"][:rows])
        else:
            assert (used >= 0).all() and (used <= it).all() and used.min() < it
    # NULL iters_used and NULL soft are allowed
    bits = np.empty((B, n), np.uint8)
    _abi.check(dec.lib.ldpc_decode(dec._h, x.ctypes.data, B, it, cl, _abi.ALGO_TANH_SP, 0, bits.ctypes.data, None,
                                   None, None))


def test_decode_bits_wifi648_equals_device_path():
    """The drop-in over a multi-chunk (648,1/2) batch equals the device-pointer decode bit for bit."""
    import ctypes
    H, _ = get_code("wifi648_12")
    cw, llr = _llr(H, 3000, 2.0, 31)
    out = ldpc_amd.decode_bits(llr.astype(np.float64), H, 20, 256, 10.0)
    rows = (3000 // 256) * 256
    dev = ldpc_amd.decode(H, torch.from_numpy(llr[:rows]).cuda(), 20, algo="tanh", clamp=10.0).cpu().numpy()
    assert np.array_equal(out[:rows], dev.astype(np.float64)) and (out[rows:] == 0).all()
    dec = ldpc_amd.get_decoder(H)
    p = dec.params(20, "tanh", 10.0)
    out2 = np.zeros_like(out)
    x = np.ascontiguousarray(llr, np.float64)  # held: a temporary's buffer would be freed before the call
    _abi.check(dec.lib.ldpc_decode_bits_host(dec._h, x.ctypes.data, rows, ctypes.byref(p), out2.ctypes.data, 333, 4))
    bad = np.nonzero((out2 != out).any(axis=1))[0]
    assert bad.size == 0, f"rows differing: {bad[:20].tolist()} (chunks {sorted(set((bad // 333).tolist()))[:10]})"


def test_belief_propagation_module_matches_reference_golden():
    d = np.load(os.path.join(GOLDEN, "bp_peg64_snr2_it10_cl10.npz"))
    BP = ldpc_amd.BeliefPropagation
    m = BP(d["H"], 10).eval().cuda()
    llr = torch.from_numpy(d["llr"]).cuda()
    x = torch.zeros(llr.shape[0], m.layer_size(), device="cuda")
    assert m.layer_size() == 96
    p1 = m(x, llr, 10).cpu().numpy()
    check_p1("module peg64_snr2_it10", p1, d["p1_f32"], d["p1_f64"], d["H"])
    m64 = m.double()
    p64 = m64(x.double(), llr.double(), 10).cpu().numpy()
    assert np.abs(p64 - d["p1_f64"]).max() <= TOL_P1_F64_VS_REF


def test_wifi648_sp_matches_reference_golden(force_generic):
    from ldpc_amd.codes import qc_expand
    d = np.load(os.path.join(GOLDEN, "bp_wifi648.npz"))
    H = qc_expand(d["base"], int(d["Z"]))
    dec = ldpc_amd.get_decoder(H)
    for tag in ("snr1", "snr2"):
        r = dec.decode(d[f"llr_{tag}"], 5, algo="tanh", clamp=10.0, soft="p1", force_generic=force_generic)
        assert np.array_equal(r["bits"], np.round(d[f"p1_f32_{tag}"]).astype(np.uint8))
        check_p1(f"wifi648 {tag} generic={force_generic}", r["soft"], d[f"p1_f32_{tag}"], d[f"p1_f64_{tag}"], H)
        r = dec.decode(d[f"llr_{tag}"].astype(np.float64), 5, algo="tanh", clamp=10.0, soft="p1", precision="f64",
                       force_generic=force_generic)
        assert np.abs(r["soft"] - d[f"p1_f64_{tag}"]).max() <= TOL_P1_F64_VS_REF


CODES = ["peg64_32", "wifi648_12", "wifi1296_23", "wifi1944_56"]


@pytest.mark.parametrize("code", CODES)
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (0.8125, 0.0), (1.0, 0.5), (0.8125, 0.5)])
def test_minsum_bit_exact_vs_oracle(code, alpha, beta, force_generic):
    """min-sum is compare/add only: GPU and oracle must agree bit for bit, soft (z) included.  Every
    normalisation the kernels instantiate: plain, alpha, beta, and alpha + beta together (NORM_BOTH)."""
    H, qc = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, 1000, 2.0 if rate < 0.6 else 4.0, seed=11, rate=rate)
    llr[0] = 0.0                       # all-zero codeword LLRs: ties everywhere
    llr[1, ::3] = 0.0
    llr[2] = np.float32(1e30)         # saturating magnitudes
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(torch.from_numpy(llr).cuda(), 25, algo="minsum", clamp=20.0, alpha=alpha, beta=beta, soft="z",
                   force_generic=force_generic)
    ref = oracle.ms_f32(H, llr, 25, 20.0, alpha, beta)
    assert np.array_equal(r["bits"].cpu().numpy(), ref["bits"])
    assert np.array_equal(r["soft"].cpu().numpy().view(np.uint32), ref["z"].view(np.uint32))


@pytest.mark.parametrize("code", CODES)
def test_sp_hard_bits_vs_oracle(code, force_generic):
    H, _ = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, 512, 1.5 if rate < 0.6 else 3.5, seed=12, rate=rate)
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(llr, 8, algo="tanh", clamp=10.0, soft="z", force_generic=force_generic)
    ref = oracle.sp_f32(H, llr, 8, 10.0, stable=True)
    mism = int((r["bits"] != ref["bits"]).sum())
    assert mism == 0, f"{mism} hard-bit mismatches"
    # soft: half-LLR z; ulp-level transcendental differences, amplified near saturation
    rel = float((np.abs(r["soft"].astype(np.float64) - ref["z"]) / np.maximum(1.0, np.abs(ref["z"]))).max())
    _log({"label": f"sp_vs_oracle {code} generic={force_generic}", "kind": "z_rel_vs_oracle", "max": rel,
          "tol": TOL_Z_REL_VS_ORACLE})
    assert rel <= TOL_Z_REL_VS_ORACLE


@pytest.mark.parametrize("B", [1, 63, 64, 65, 1000])
def test_ragged_batches(B):
    H, _ = get_code("wifi648_12")
    cw, llr = _llr(H, B, 2.0, seed=B)
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(llr, 10, algo="minsum", clamp=20.0, soft="z")
    ref = oracle.ms_f32(H, llr, 10, 20.0)
    assert np.array_equal(r["bits"], ref["bits"]) and np.array_equal(r["soft"], ref["z"])


def test_zero_iterations_and_empty_batch():
    H, _ = get_code("peg64_32")
    cw, llr = _llr(H, 16, 2.0, seed=3)
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(llr, 0, algo="tanh", clamp=10.0, soft="z")
    assert np.array_equal(r["soft"], (np.float32(0.5) * -llr).astype(np.float32))
    r = dec.decode(np.zeros((0, 64), np.float32), 5)
    assert r["bits"].shape == (0, 64)


def test_count_errors_and_awgn():
    lib = _abi.load()
    B, n = 3000, 648
    bits = torch.randint(0, 2, (B, n), dtype=torch.uint8, device="cuda")
    ref = torch.randint(0, 2, (B, n), dtype=torch.uint8, device="cuda")
    ref[:100] = bits[:100]
    counts = torch.zeros(3, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    _abi.check(lib.ldpc_count_errors(bits.data_ptr(), ref.data_ptr(), B, n, 324, counts.data_ptr(), st))
    b, r = bits.cpu().numpy(), ref.cpu().numpy()
    assert counts.cpu().tolist() == [int((b[:, :324] != r[:, :324]).sum()), int((b != r).any(1).sum()), B]
    llr = torch.empty((B, n), dtype=torch.float32, device="cuda")
    sigma = 0.8
    _abi.check(lib.ldpc_awgn_llr(ref.data_ptr(), llr.data_ptr(), B, n, sigma, 1234, 0, st))
    y = (-llr * sigma**2 / 2).cpu().numpy()
    noise = y - (1 - 2 * r.astype(np.float64))
    assert abs(noise.mean()) < 0.01 and abs(noise.std() - sigma) < 0.01
    # a shard's LLRs do not depend on the shard split
    llr2 = torch.empty((B - 1000, n), dtype=torch.float32, device="cuda")
    _abi.check(lib.ldpc_awgn_llr(ref[1000:].data_ptr(), llr2.data_ptr(), B - 1000, n, sigma, 1234, 1000, st))
    assert torch.equal(llr2, llr[1000:])


# ---------------------------------------------------------------- QC register kernel specifics
QC_CODES = ["wifi648_12", "wifi1296_23", "wifi1944_56"]  # Z = 81: sliced kernels (qc_sl.hip)
QC_SP_CODES = QC_CODES


@pytest.mark.parametrize("code", QC_SP_CODES)
def test_qc_kernel_is_selected(code):
    H, qc = get_code(code)
    assert ldpc_amd.get_decoder(H).qc_z == qc.Z


@pytest.mark.parametrize("code", QC_CODES)
@pytest.mark.parametrize("snr", [1.0, 2.5, 4.0])
@pytest.mark.parametrize("alpha,beta", [(0.8125, 0.0), (1.0, 0.0), (1.0, 0.5), (0.8125, 0.5)])
def test_qc_early_stop_vs_oracle(code, snr, alpha, beta):
    """Early-stop min-sum, every normalisation (these kernels come from qc_es.hip): iteration counts,
    bits and z bitwise equal to the oracle; 777 codewords leave the last wave's second codeword empty."""
    H, qc = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, 777, snr + (2.0 if rate > 0.6 else 0.0), seed=int(snr * 10), rate=rate)
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(torch.from_numpy(llr).cuda(), 20, algo="minsum", clamp=20.0, alpha=alpha, beta=beta,
                   early_stop=True, soft="z", want_iters=True)
    ref = oracle.ms_f32(H, llr, 20, 20.0, alpha, beta, early_stop=True)
    assert np.array_equal(r["iters_used"].cpu().numpy(), ref["iters_used"])
    assert np.array_equal(r["bits"].cpu().numpy(), ref["bits"])
    assert np.array_equal(r["soft"].cpu().numpy().view(np.uint32), ref["z"].view(np.uint32))


@pytest.mark.parametrize("code", QC_CODES)
@pytest.mark.parametrize("early", [False, True])
@pytest.mark.parametrize("beta", [0, 1])
def test_qc_quantized_minsum_vs_oracle(code, early, beta):
    H, qc = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, 500, 3.0 if rate < 0.6 else 4.5, seed=21 + beta, rate=rate)
    qstep = np.float32(0.75)
    qinv = np.float32(1.0) / qstep
    q = np.clip(np.rint(llr * qinv), -15, 15).astype(np.int8)
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(llr, 20, algo="qminsum", qmax=15, app_max=127, qstep=float(qstep), beta=float(beta),
                   early_stop=early, soft="z", want_iters=True)
    ref = oracle.qms(H, q, 20, 15, 127, beta, early_stop=early)
    assert np.array_equal(r["iters_used"], ref["iters_used"])
    assert np.array_equal(r["bits"], ref["bits"])
    assert np.array_equal(r["soft"], (0.5 * ref["app"]).astype(np.float32))


@pytest.mark.parametrize("code", QC_CODES)
@pytest.mark.parametrize("qmax,app_max,qstep,beta", [(7, 31, 0.5, 2), (127, 2047, 0.125, 3), (31, 32767, 1.0, 0),
                                                     (3, 3, 2.0, 1)])
def test_qc_quantized_minsum_quantizer_ranges(code, qmax, app_max, qstep, beta):
    """Quantizer widths other than 5 bit: the message / APP saturations, offsets up to beta = 3 and
    app_max above every reachable posterior (the packed kernel's fp16 halves stay exact: |L + sum c2v| <=
    (1 + d_v) qmax <= 1651 < 2048) — bits, APP and iteration counts bitwise vs the oracle."""
    H, qc = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, 300, 3.0 if rate < 0.6 else 4.5, seed=5 + qmax, rate=rate)
    qs = np.float32(qstep)
    q = np.clip(np.rint(llr * (np.float32(1.0) / qs)), -qmax, qmax).astype(np.int32)
    dec = ldpc_amd.get_decoder(H)
    for early in (False, True):
        r = dec.decode(llr, 12, algo="qminsum", qmax=qmax, app_max=app_max, qstep=float(qs), beta=float(beta),
                       early_stop=early, soft="z", want_iters=True)
        ref = oracle.qms(H, q, 12, qmax, app_max, beta, early_stop=early)
        assert np.array_equal(r["iters_used"], ref["iters_used"])
        assert np.array_equal(r["bits"], ref["bits"])
        assert np.array_equal(r["soft"], (0.5 * ref["app"]).astype(np.float32))


def test_degenerate_graph_empty_row_and_column():
    """An all-zero row and column of H (the reference accepts any binary H, masking.py:12)."""
    H, _ = get_code("peg64_32")
    H = np.concatenate([H, np.zeros((1, 64), H.dtype)], axis=0)     # empty check
    H = np.concatenate([H, np.zeros((33, 1), H.dtype)], axis=1)     # unconnected variable
    rng = np.random.default_rng(4)
    llr = rng.normal(2.0, 2.0, size=(100, 65)).astype(np.float32)
    dec = ldpc_amd.get_decoder(H)
    for algo, ref in (("minsum", oracle.ms_f32(H, llr, 7, 20.0)), ("tanh", oracle.sp_f32(H, llr, 7, 20.0, stable=True))):
        r = dec.decode(llr, 7, algo=algo, clamp=20.0, soft="z")
        assert np.array_equal(r["bits"], ref["bits"])


@pytest.mark.parametrize("name,B,iters,ebn0", [("dvbs2_12", 32, 50, 0.9), ("dvbs2s_12", 6, 12, 3.0)])
def test_dvbs2_minsum_bit_exact_and_sp_bits(name, B, iters, ebn0):
    """BASELINE config [4]'s code (EN 302 307 rate 1/2, codes.dvbs2_12) at its 50 iterations on 32 codewords,
    and the shaped stand-in: min-sum bits and z bitwise vs the oracle (plain min-sum as config [4] runs it, and
    normalised), tanh-SP bits identical and z within the oracle tolerance; the reference cannot instantiate
    n = 64800 (dense E x E masks, masking.py:36-38), so parity against the reference is unpinned here."""
    from ldpc_amd.codes import IRAEncoder
    c, _ = get_code(name)
    rng = np.random.default_rng(9)
    cw = IRAEncoder(c).encode(rng.integers(0, 2, size=(B, c.k)))
    sigma = np.sqrt(1.0 / (2 * 0.5 * 10 ** (ebn0 / 10)))  # EN 302 307 at 0.9 dB: in the waterfall (31/32 decode)
    llr = (-2.0 * ((1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)) / sigma**2).astype(np.float32)
    dec = ldpc_amd.get_decoder(c)
    x = torch.from_numpy(llr).cuda()
    for alpha in (1.0, 0.75):
        r = dec.decode(x, iters, algo="minsum", alpha=alpha, clamp=20.0, soft="z")
        ref = oracle.ms_f32(c, llr, iters, 20.0, alpha, 0.0)
        assert np.array_equal(r["bits"].cpu().numpy(), ref["bits"])
        assert np.array_equal(r["soft"].cpu().numpy().view(np.uint32), ref["z"].view(np.uint32))
    r = dec.decode(x, iters, algo="tanh", clamp=10.0, soft="z")
    ref = oracle.sp_f32(c, llr, iters, 10.0, stable=True)
    # codewords the oracle decodes (zero syndrome): bits identical, z to the oracle tolerance; on decoding
    # failures 50 iterations amplify ulp-level exp/log differences, so only their count is compared
    par = np.add.reduceat(ref["bits"][:, c.col_idx].astype(np.int64), c.row_ptr[:-1], axis=1) % 2
    ok = ~par.any(axis=1)
    got_bits = r["bits"].cpu().numpy()
    assert ok.sum() >= B // 4 and np.array_equal(got_bits[ok], ref["bits"][ok])
    gpar = np.add.reduceat(got_bits[:, c.col_idx].astype(np.int64), c.row_ptr[:-1], axis=1) % 2
    assert abs(int((~gpar.any(axis=1)).sum()) - int(ok.sum())) <= max(1, B // 16)
    z = r["soft"].cpu().numpy().astype(np.float64)[ok]
    rel = np.abs(z - ref["z"][ok]) / np.maximum(1.0, np.abs(ref["z"][ok]))
    _log({"label": f"sp_vs_oracle {name} {iters} it decoded", "kind": "z_rel_vs_oracle", "max": float(rel.max())})
    assert rel.max() <= TOL_Z_REL_VS_ORACLE


@pytest.mark.parametrize("code", ["peg64_32", "wifi648_12", "wifi1944_56"])
@pytest.mark.parametrize("algo", ["minsum", "tanh"])
def test_generic_early_stop_vs_oracle(code, algo):
    H, _ = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, 301, 2.5 if rate < 0.6 else 4.5, seed=31, rate=rate)
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(llr, 20, algo=algo, clamp=20.0, early_stop=True, force_generic=True, want_iters=True, soft="z")
    if algo == "minsum":
        ref = oracle.ms_f32(H, llr, 20, 20.0, early_stop=True)
        assert np.array_equal(r["soft"].view(np.uint32), ref["z"].view(np.uint32))
    else:
        ref = oracle.sp_f32(H, llr, 20, 20.0, early_stop=True, stable=True)
    assert np.array_equal(r["iters_used"], ref["iters_used"])
    assert np.array_equal(r["bits"], ref["bits"])
    assert (ref["iters_used"] < 20).any()          # the test exercises convergence


@pytest.mark.parametrize("code", QC_SP_CODES)
@pytest.mark.parametrize("B", [1, 1001])
def test_qc_sp_equals_generic_sp_bitwise(code, B):
    """The on-chip tanh-SP kernel performs the generic kernels' operations in the same order with the
    same tanhf/logf, so z (and p1) agree bit for bit; both match the oracle's hard bits."""
    H, qc = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, B, 1.5 if rate < 0.6 else 3.0, seed=21, rate=rate)
    llr[0, ::5] = 0.0
    if B > 2:
        llr[1] = np.float32(60.0)
    dec = ldpc_amd.get_decoder(H)
    x = torch.from_numpy(llr).cuda()
    for soft in ("z", "p1"):
        a = dec.decode(x, 30, algo="tanh", clamp=10.0, soft=soft)
        b = dec.decode(x, 30, algo="tanh", clamp=10.0, soft=soft, force_generic=True)
        assert torch.equal(a["bits"], b["bits"])
        assert torch.equal(a["soft"].view(torch.int32), b["soft"].view(torch.int32))
    r = dec.decode(x, 30, algo="tanh", clamp=10.0, want_iters=True)
    assert bool((r["iters_used"] == 30).all())


@pytest.mark.parametrize("code", ["wifi648_12", "wifi1296_23", "wifi1944_56"])
@pytest.mark.parametrize("B", [1, 2, 777])
def test_qc_sp_early_stop_equals_generic_bitwise(code, B):
    """tanh-SP with early termination in the register kernels (Z <= 64: k_qc_sp_st; Z = 81: the sliced
    k_qc_sp_sl, whose three waves agree through LDS): iteration counts, bits and z equal the generic
    kernels' (whose counts equal the oracle's, test_generic_early_stop_vs_oracle), including codeword pairs
    that stop at different iterations and an odd batch."""
    H, qc = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, B, 2.0 if rate < 0.6 else (3.5 if rate < 0.8 else 4.2), seed=51 + B, rate=rate)
    if B > 2:
        llr[2] = np.float32(-50.0) * (1 - 2 * cw[2])     # converges at the first check
    dec = ldpc_amd.get_decoder(H)
    assert dec.qc_z == qc.Z
    x = torch.from_numpy(llr).cuda()
    a = dec.decode(x, 20, algo="tanh", clamp=10.0, early_stop=True, want_iters=True, soft="z")
    b = dec.decode(x, 20, algo="tanh", clamp=10.0, early_stop=True, want_iters=True, soft="z", force_generic=True)
    assert torch.equal(a["iters_used"], b["iters_used"])
    assert torch.equal(a["bits"], b["bits"])
    assert torch.equal(a["soft"].view(torch.int32), b["soft"].view(torch.int32))
    if B > 2:
        u = a["iters_used"].cpu().numpy()
        assert (u < 20).any() and len(np.unique(u)) > 1   # early exits at several iterations


@pytest.mark.parametrize("code", ["wifi648_12", "dvbs2s_12"])
def test_cache_resident_chunks_match_single_pass(code, monkeypatch):
    """The generic path decodes in Infinity-Cache-sized chunks (LDPC_CACHE_BUDGET_MB).  A tiny budget forces
    64-codeword chunks (narrow 64-lane tiles) plus a ragged tail; results must equal the single-pass decode
    bit for bit and the oracle's (min-sum bitwise, early-stop iteration counts included)."""
    if code == "dvbs2s_12":
        from ldpc_amd.codes import IRAEncoder, dvbs2_shaped
        H = dvbs2_shaped()
        rng = np.random.default_rng(5)
        cw = IRAEncoder(H).encode(rng.integers(0, 2, size=(133, H.k)))
        sigma = np.sqrt(1.0 / (2 * 0.5 * 10 ** (1.2 / 10)))
        llr = (-2.0 * ((1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)) / sigma**2).astype(np.float32)
        iters = 6
    else:
        H, _ = get_code(code)
        _, llr = _llr(H, 301, 2.0, seed=41)
        iters = 20
    dec = ldpc_amd.get_decoder(H)
    x = torch.from_numpy(llr).cuda()
    out = {}
    for budget in ("0", "1"):
        monkeypatch.setenv("LDPC_CACHE_BUDGET_MB", budget)
        out[budget] = [dec.decode(x, iters, algo="minsum", clamp=20.0, early_stop=True, force_generic=True,
                                  want_iters=True, soft="z"),
                       dec.decode(x, iters, algo="tanh", clamp=10.0, force_generic=True, soft="p1")]
    for a, b in zip(out["0"], out["1"]):
        for k in ("bits", "soft", "iters_used"):
            if a.get(k) is None:
                assert b.get(k) is None
                continue
            assert torch.equal(a[k].view(torch.int32) if a[k].dtype == torch.float32 else a[k],
                               b[k].view(torch.int32) if b[k].dtype == torch.float32 else b[k]), k
    if code == "wifi648_12":
        ref = oracle.ms_f32(H, llr, iters, 20.0, early_stop=True)
        r = out["1"][0]
        assert np.array_equal(r["iters_used"].cpu().numpy(), ref["iters_used"])
        assert np.array_equal(r["soft"].cpu().numpy().view(np.uint32), ref["z"].view(np.uint32))
        r64 = dec.decode(llr.astype(np.float64), 5, algo="tanh", clamp=10.0, precision="f64", soft="p1",
                         force_generic=True)
        monkeypatch.setenv("LDPC_CACHE_BUDGET_MB", "0")
        r64b = dec.decode(llr.astype(np.float64), 5, algo="tanh", clamp=10.0, precision="f64", soft="p1",
                          force_generic=True)
        assert np.array_equal(r64["soft"], r64b["soft"])


def test_side_stream_and_device_checks():
    """decode(stream=side) is ordered after the producer on the current stream and equals the default-stream
    decode; a device mismatch raises instead of launching on foreign pointers."""
    H, _ = get_code("wifi648_12")
    cw, llr = _llr(H, 300, 2.0, seed=8)
    dec = ldpc_amd.get_decoder(H)
    src = torch.from_numpy(llr).cuda()
    want = dec.decode(src, 10, algo="minsum", clamp=20.0, soft="z")
    side = torch.cuda.Stream()
    for _ in range(3):
        x = src * 1.0                      # produced on the current stream just before the decode
        r = dec.decode(x, 10, algo="minsum", clamp=20.0, soft="z", stream=side)
        del x                              # recycled only after the side stream has read it
        side.synchronize()
        assert torch.equal(r["bits"], want["bits"]) and torch.equal(r["soft"], want["soft"])
    r = dec.decode(src, 10, algo="minsum", clamp=20.0, soft="z", stream=side.cuda_stream)  # a raw handle
    side.synchronize()
    assert torch.equal(r["bits"], want["bits"]) and torch.equal(r["soft"], want["soft"])
    with pytest.raises(TypeError):
        dec.decode(src, 10, stream="side")
    # weighted and initial-message decodes on the side stream: the weights (uploaded on the current stream)
    # and the caller's x0 are held until the side stream has read them
    g = dec.graph
    rng = np.random.default_rng(3)
    w = {"vn": rng.uniform(0.5, 1.5, (6, dec.weights_per_iter)).astype(np.float32),
         "llr": rng.uniform(0.5, 1.5, (6, g.n)).astype(np.float32)}
    want_w = dec.decode(src, 6, algo="tanh", soft="z", weights=w)
    want_x = dec.decode(src, 6, algo="tanh", soft="z", x0=torch.full((300, g.E), 0.25, device="cuda"))
    for _ in range(3):
        x0 = torch.full((300, g.E), 0.25, device="cuda")
        rw = dec.decode(src, 6, algo="tanh", soft="z", weights=w, stream=side)
        rx = dec.decode(src, 6, algo="tanh", soft="z", x0=x0, stream=side)
        del x0
        torch.empty((300, g.E), device="cuda").fill_(7.0)   # would reuse x0's block if it were released early
        side.synchronize()
        assert torch.equal(rw["soft"], want_w["soft"]) and torch.equal(rx["soft"], want_x["soft"])
    with pytest.raises(ValueError):
        ldpc_amd.decode(H, src, 5, device=src.device.index + 1)


def test_quantized_minsum_rejects_fractional_offset_and_alpha():
    """QMIN_SUM is integer offset min-sum: beta must be a whole number and alpha 1 (ldpc_abi.h)."""
    H, _ = get_code("wifi648_12")
    dec = ldpc_amd.get_decoder(H)
    x = torch.zeros((4, 648), device="cuda")
    for kw in (dict(beta=0.5), dict(alpha=0.75), dict(beta=-1.0)):
        with pytest.raises(_abi.LdpcError):
            dec.decode(x, 3, algo="qminsum", **kw)
    dec.decode(x, 3, algo="qminsum", beta=1.0)


@pytest.mark.parametrize("code", ["wifi648_12", "wifi1296_23"])
@pytest.mark.parametrize("B", [1, 2, 3, 5, 127])
@pytest.mark.parametrize("early", [False, True])
def test_packed_quantized_ragged_batches(code, B, early):
    """The packed 5-bit kernel holds 2 codewords per lane (4 per wave at Z = 27, 2 at Z = 54): batches that do
    not fill the last lane group, its high fp16 half, or the last wave must decode exactly like the oracle
    (bits, z, iteration counts) and write nothing past row B - 1."""
    H, _ = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, B, 2.5 if rate < 0.6 else 4.0, seed=300 + B, rate=rate)
    q = np.clip(np.rint(llr), -15, 15).astype(np.int8)
    dec = ldpc_amd.get_decoder(H)
    x = torch.from_numpy(llr).cuda()
    r = dec.decode(x, 20, algo="qminsum", qmax=15, app_max=127, qstep=1.0, early_stop=early, soft="z", want_iters=True)
    ref = oracle.qms(H, q, 20, 15, 127, 0, early_stop=early)
    assert np.array_equal(r["bits"].cpu().numpy(), ref["bits"])
    assert np.array_equal(r["soft"].cpu().numpy(), (0.5 * ref["app"]).astype(np.float32))
    assert np.array_equal(r["iters_used"].cpu().numpy(), ref["iters_used"])
    # no writes past the batch: decode into a larger buffer through the ABI and check the guard rows
    p = dec.params(20, "qminsum", 15.0, 1.0, 0.0, early, "f32", "z", device_ptrs=True)
    bits = torch.full((B + 4, H.shape[1]), 7, dtype=torch.uint8, device="cuda")
    soft = torch.full((B + 4, H.shape[1]), 7.0, dtype=torch.float32, device="cuda")
    used = torch.full((B + 4,), 77, dtype=torch.int32, device="cuda")
    ws = torch.empty((max(dec.workspace_bytes(B, p), 1),), dtype=torch.uint8, device="cuda")
    _abi.check(dec.lib.ldpc_decode_ex(dec._h, x.data_ptr(), B, p, bits.data_ptr(), soft.data_ptr(), used.data_ptr(),
                                      ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert (bits[B:] == 7).all() and (soft[B:] == 7.0).all() and (used[B:] == 77).all()
    assert np.array_equal(bits[:B].cpu().numpy(), ref["bits"])


@pytest.mark.parametrize("code", ["wifi648_12", "wifi1296_23"])
def test_packed_quantized_io_alignment(code):
    """LLR and bit buffers at any alignment (the ABI takes plain pointers: views into larger buffers), a ragged
    B, bits only and with soft output: bit-identical to the oracle, and nothing outside [bits, bits + B * n)
    is written.  (16-byte vector loads / stores staged through LDS were measured 1-2 % slower for this kernel,
    DESIGN.md §3.3, so there is one per-element path.)"""
    H, _ = get_code(code)
    n = H.shape[1]
    B = 37
    cw, llr = _llr(H, B, 3.0, seed=77, rate=1 - H.shape[0] / n)
    q = np.clip(np.rint(llr), -15, 15).astype(np.int8)
    dec = ldpc_amd.get_decoder(H)
    for early in (False, True):
        ref = oracle.qms(H, q, 20, 15, 127, 0, early_stop=early)
        for xoff, boff, soft in ((0, 0, "none"), (1, 0, "none"), (0, 3, "none"), (2, 9, "z"), (0, 0, "z")):
            xs = torch.zeros(B * n + 8, dtype=torch.float32, device="cuda")
            xs[xoff:xoff + B * n] = torch.from_numpy(llr.reshape(-1)).cuda()
            bs = torch.full((B * n + 64,), 7, dtype=torch.uint8, device="cuda")
            sf = torch.zeros((B, n), dtype=torch.float32, device="cuda")
            p = dec.params(20, "qminsum", 15.0, 1.0, 0.0, early, "f32", soft, device_ptrs=True)
            ws = torch.empty((max(dec.workspace_bytes(B, p), 1),), dtype=torch.uint8, device="cuda")
            _abi.check(dec.lib.ldpc_decode_ex(dec._h, xs.data_ptr() + 4 * xoff, B, p, bs.data_ptr() + boff,
                                              sf.data_ptr() if soft != "none" else 0, 0, ws.data_ptr(), ws.numel(),
                                              torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            got = bs.cpu().numpy()
            assert (got[:boff] == 7).all() and (got[boff + B * n:] == 7).all(), (xoff, boff, soft)
            assert np.array_equal(got[boff:boff + B * n].reshape(B, n), ref["bits"]), (xoff, boff, soft, early)
            if soft != "none":
                assert np.array_equal(sf.cpu().numpy(), (0.5 * ref["app"]).astype(np.float32))


def test_decode_bits_reference_receiver_chain_golden():
    """The drop-in on the reference's own receiver chain (tests/golden/e2e_wifi648_qpsk_ofdm.npz: the reference's
    bits -> encode_bits -> modulate_bits -> gen_data's 32-point OFDM over AWGN -> demodulate_signal LLRs ->
    decode_bits(llrs, H, 50, 40, 10), evaluate_snr.py's pipeline) on (648,1/2) in the waterfall: the float64 output
    equals the reference's exactly — decoded and failing rows, and the zero tail rows 80..95."""
    from ldpc_amd.codes import qc_expand
    d = np.load(os.path.join(GOLDEN, "e2e_wifi648_qpsk_ofdm.npz"))
    H = qc_expand(d["base"], int(d["Z"]))
    for snr in d["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        out = ldpc_amd.decode_bits(d[f"llrs_{tag}"], H, int(d["iters"]), int(d["batch_size"]), int(d["clamp"]))
        assert out.dtype == np.float64 and out.shape == d[f"out_{tag}"].shape
        assert np.array_equal(out, d[f"out_{tag}"]), tag


def test_decode_bits_reference_quantized_chain_golden():
    """The drop-in on the reference's quantized receiver chain (tests/golden/e2e_quantized.npz: gen_qdata's ADC,
    evaluate_quantized.py's pipeline, clamp 20): (64,32) at 3 iterations with the evaluator's 3-bit ADC, (648,1/2)
    at 50 with a 5-bit ADC — LLRs with exact zeros; the float64 output equals the reference's exactly."""
    d = np.load(os.path.join(GOLDEN, "e2e_quantized.npz"))
    for name in ("peg64", "wifi648"):
        iters, bs, clamp = (int(x) for x in d[f"cfg_{name}"][:3])
        out = ldpc_amd.decode_bits(d[f"llrs_{name}"], d[f"H_{name}"].astype(np.int64), iters, bs, clamp)
        assert out.dtype == np.float64 and np.array_equal(out, d[f"out_{name}"]), name


def test_decode_llr_sign_convention():
    """decode(..., llr_sign="p0/p1") takes the communications convention (positive = bit 0): the same bits
    as the reference convention on the negated input."""
    H, _ = get_code("wifi648_12")
    cw, llr = _llr(H, 64, 2.0, seed=3)
    a = ldpc_amd.decode(H, llr, 10, algo="minsum", clamp=20.0)
    b = ldpc_amd.decode(H, -llr, 10, algo="minsum", clamp=20.0, llr_sign="p0/p1")
    c = ldpc_amd.decode(H, torch.from_numpy(-llr).cuda(), 10, algo="minsum", clamp=20.0, llr_sign="p0/p1").cpu().numpy()
    assert np.array_equal(a, b) and np.array_equal(a, c)
    with pytest.raises(ValueError):
        ldpc_amd.decode(H, llr, 10, llr_sign="bogus")


@pytest.mark.parametrize("code", ["peg64_32", "wifi648_12", "wifi1296_23", "wifi1944_56"])
def test_tanh_zero_llr_rows_exact(code, force_generic):
    """All-zero LLR rows through tanh-SP (register / sliced and generic kernels): the reference gives z = 0
    exactly (tanh(0) = 0 zeroes every product; p1 = 0.5 rounds to bit 0); the (D, S) form keeps D == S
    exactly for a = 1, so the GPU must return exact zeros too, and equal the oracle's bits elsewhere."""
    H, _ = get_code(code)
    rate = 1 - H.shape[0] / H.shape[1]
    cw, llr = _llr(H, 130, 1.5 if rate < 0.6 else 3.5, seed=77, rate=rate)
    llr[:3] = 0.0
    dec = ldpc_amd.get_decoder(H)
    r = dec.decode(torch.from_numpy(llr).cuda(), 12, algo="tanh", clamp=10.0, soft="z", force_generic=force_generic)
    z = r["soft"].cpu().numpy()
    assert np.all(z[:3] == 0.0) and not r["bits"][:3].cpu().numpy().any()
    ref = oracle.sp_f32(H, llr, 12, 10.0, stable=True)
    assert np.array_equal(r["bits"].cpu().numpy(), ref["bits"])


@pytest.mark.parametrize("name,iters", [("wifi648_12", 50), ("wifi1296_23", 20), ("wifi1944_56", 10)])
def test_decode_bits_dropin_long_reference_goldens(name, iters):
    """The drop-in itself (decode_bits from host float64, ofdm_functions.py:131-163) on the reference runs at
    the drop-in's / BASELINE configs' iteration counts: every decoded row's bits equal the reference's fp32
    decode_bits bits (np.round(p1)); the ragged tail (N % batch_size) stays 0."""
    from ldpc_amd.codes import qc_expand
    d = np.load(os.path.join(GOLDEN, f"bp_{name}_sp_it{iters}.npz"))
    H = qc_expand(d["base"], int(d["Z"]))
    for snr in d["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        llr = d[f"llr_{tag}"].astype(np.float64)
        bs = max(1, llr.shape[0] // 3)
        out = ldpc_amd.decode_bits(llr, H, iters, bs, float(d["clamp"]))
        rows = (llr.shape[0] // bs) * bs
        assert out.dtype == np.float64
        assert np.array_equal(out[:rows], np.round(d[f"p1_f32_{tag}"][:rows]).astype(np.float64))
        assert not out[rows:].any()


@pytest.mark.parametrize("code", ["peg64_32", "wifi648_12"])
def test_clustered_zero_llrs_vs_reference_golden(code):
    """Clustered exact-zero LLRs through the reference (tests/golden/bp_zeros.npz, 1/2/3/5 iterations, clamp 10
    and 20): the GPU (the register kernel's a == 1 pass on (648,1/2), the generic kernels on both) meets the
    reference as the oracle does (softparity.check_zeros_golden: exact zeros where the reference's are, its
    fp32 bits outside the rounding band), and the kernel families agree bit for bit."""
    from softparity import check_zeros_golden
    d = np.load(os.path.join(GOLDEN, "bp_zeros.npz"))
    H = np.asarray(get_code(code)[0])
    dec = ldpc_amd.get_decoder(H)
    x = torch.from_numpy(d[f"{code}_llr"]).cuda()
    for it in (1, 2, 3, 5):
        for cl in (10, 20):
            tag = f"{code}_it{it}_cl{cl}"
            a = dec.decode(x, it, algo="tanh", clamp=float(cl), soft="z")
            g = dec.decode(x, it, algo="tanh", clamp=float(cl), soft="z", force_generic=True)
            assert torch.equal(a["bits"], g["bits"]) and torch.equal(a["soft"].view(torch.int32), g["soft"].view(torch.int32)), tag
            check_zeros_golden(f"gpu zeros {code}", a["bits"].cpu().numpy(), a["soft"].cpu().numpy(), d, tag)


@pytest.mark.parametrize("code,early", [("wifi648_12", True), ("wifi1296_23", False), ("wifi1296_23", True),
                                        ("wifi1944_56", False), ("wifi1944_56", True)])
def test_zero_llr_pass_equals_generic_bitwise(code, early):
    """Every tanh-SP register kernel's a == 1 pass (PASS 2: the waves / units whose LLRs hold an exact zero)
    against the generic kernels bit for bit — bits, z and iteration counts — on a batch where about half the
    codewords carry erasures (so both passes of one launch write outputs), fixed count and early stop."""
    H = np.asarray(get_code(code)[0])
    dec = ldpc_amd.get_decoder(H)
    rate = 1 - H.shape[0] / H.shape[1]
    _, x = _llr(H, 37, 3.0, seed=17, rate=rate)
    rng = np.random.default_rng(5)
    er = rng.random(x.shape) < 0.04
    er[::2] = False                                   # even rows: no erasure (the plain pass)
    x[er] = 0.0
    xt = torch.from_numpy(x).cuda()
    kw = dict(algo="tanh", clamp=20.0, soft="z", early_stop=early, want_iters=True)
    a = dec.decode(xt, 20, **kw)
    g = dec.decode(xt, 20, force_generic=True, **kw)
    assert torch.equal(a["bits"], g["bits"])
    assert torch.equal(a["soft"].view(torch.int32), g["soft"].view(torch.int32))
    assert torch.equal(a["iters_used"], g["iters_used"])
