"""Pin the CPU oracle against the reference's own outputs (tests/golden, made by make_golden.py from
pytorch/bp/bp.py + ofdm_functions.decode_bits run in the build container)."""
import glob
import os

import numpy as np
import pytest

import oracle
import numpy_ref
from conftest import GOLDEN

PEG_FILES = sorted(glob.glob(os.path.join(GOLDEN, "bp_peg64_snr*.npz")))

# tolerances (documented in DESIGN.md "Parity"): fp32 soft output p1 vs the reference's fp32 module;
# fp64 vs the reference module after .double().
TOL_P1_F32 = 5e-6
TOL_P1_F64 = 1e-12


def test_golden_files_present():
    assert len(PEG_FILES) == 15


@pytest.mark.parametrize("path", PEG_FILES, ids=lambda p: os.path.basename(p))
def test_oracle_sp_f32_matches_reference(path):
    d = np.load(path)
    r = oracle.sp_f32(d["H"], d["llr"], int(d["iters"]), float(d["clamp"]))
    assert np.array_equal(r["bits"], d["bits_f32"])
    assert np.abs(r["p1"] - d["p1_f32"]).max() <= TOL_P1_F32


@pytest.mark.parametrize("path", PEG_FILES, ids=lambda p: os.path.basename(p))
def test_oracle_sp_f64_matches_reference(path):
    d = np.load(path)
    r = oracle.sp_f64(d["H"], d["llr"].astype(np.float64), int(d["iters"]), float(d["clamp"]))
    assert np.array_equal(r["bits"], d["bits_f64"])
    assert np.abs(r["p1"] - d["p1_f64"]).max() <= TOL_P1_F64


def test_oracle_c2v_trace_matches_reference():
    """Per-iteration check-order messages x (bp/bp.py:46-47): pins edge numbering and the CV update."""
    d = np.load(os.path.join(GOLDEN, "bp_peg64_trace.npz"))
    r = oracle.sp_f32(d["H"], d["llr"], 5, 10.0, trace=True)
    assert r["trace"].shape == d["x_f32"].shape
    assert np.abs(r["trace"] - d["x_f32"]).max() <= 2e-5   # c2v values are up to 16.6: ~1 ulp-level
    # in fp64 the restatement follows the reference to rounding
    z64 = numpy_ref.sp(d["H"], d["llr"].astype(np.float64), 5, 10.0)
    p1 = 1 - 1 / (1 + np.exp(-z64))
    assert np.abs(p1 - d["p1_f64"]).max() <= 1e-12


def test_oracle_decode_bits_boundary():
    """decode_bits (ofdm_functions.py:131-163): float64 output, ragged tail rows stay 0."""
    d = np.load(os.path.join(GOLDEN, "decode_bits_peg64.npz"))
    out = d["out"]
    assert str(d["out_dtype"]) == "float64"
    N, bs = out.shape[0], int(d["batch_size"])
    rows = (N // bs) * bs
    r = oracle.sp_f32(d["H"], d["llrs"].astype(np.float32), int(d["iters"]), float(d["clamp"]))
    assert np.array_equal(r["bits"][:rows].astype(np.float64), out[:rows])
    assert not out[rows:].any()


def test_oracle_wifi648_matches_reference():
    from ldpc_amd.codes import qc_expand
    d = np.load(os.path.join(GOLDEN, "bp_wifi648.npz"))
    H = qc_expand(d["base"], int(d["Z"]))
    for tag in ("snr1", "snr2"):
        r32 = oracle.sp_f32(H, d[f"llr_{tag}"], 5, 10.0)
        r64 = oracle.sp_f64(H, d[f"llr_{tag}"].astype(np.float64), 5, 10.0)
        assert np.array_equal(r32["bits"], np.round(d[f"p1_f32_{tag}"]).astype(np.uint8))
        assert np.array_equal(r64["bits"], np.round(d[f"p1_f64_{tag}"]).astype(np.uint8))
        assert np.abs(r32["p1"] - d[f"p1_f32_{tag}"]).max() <= TOL_P1_F32
        assert np.abs(r64["p1"] - d[f"p1_f64_{tag}"]).max() <= TOL_P1_F64


def test_hard_decision_threshold():
    """bit = np.round(1 - sigmoid(z)) in fp32 <=> z <= -1.7881392e-07 (0xb43fffff), measured on torch 2.10."""
    thr = np.array([0xB43FFFFF], np.uint32).view(np.float32)[0]
    assert thr == np.float32(-1.7881392e-07)
    H = np.array([[1, 1]])
    # iters=0: z = -0.5*llr, so llr = -2z probes the decision directly
    zs = np.array([[thr, thr], [np.nextafter(thr, np.float32(0)), 0.0]], np.float32)
    r = oracle.sp_f32(H, (-2 * zs).astype(np.float32), 0, 10.0)
    assert r["bits"].tolist() == [[1, 1], [0, 0]]


def test_weighted_oracle_matches_reference_golden():
    """Weighted BP (bp_vc.py:19,24 with random non-unit weights set in the reference module): the oracle
    on the compact weight layout reproduces the reference's fp64 and fp32 p1."""
    from ldpc_amd.codes import Graph
    d = np.load(os.path.join(GOLDEN, "bp_weighted_peg64.npz"))
    H, iters, clamp = d["H"], int(d["iters"]), float(d["clamp"])
    g = Graph.from_H(H)
    w = g.compact_weights([d[f"input_weight{i}"] for i in range(iters)], [d[f"llr_weight{i}"] for i in range(iters)],
                          d["final_input_weight"], d["final_llr_weight"])
    # every reference weight on the mask is carried over (and nothing off it)
    tgt, src, pos = g.vn_weight_index()
    assert np.count_nonzero(d["input_weight0"]) == len(pos)
    for tag in ("snr1", "snr3"):
        llr = d[f"llr_{tag}"]
        r64 = oracle.sp_f64(H, llr.astype(np.float64), iters, clamp, weights=w)
        assert np.abs(r64["p1"] - d[f"p1_f64_{tag}"]).max() < 1e-12
        r32 = oracle.sp_f32(H, llr, iters, clamp, weights=w)
        assert np.abs(r32["p1"] - d[f"p1_f32_{tag}"]).max() < 5e-5
        assert (r32["bits"] != np.round(d[f"p1_f32_{tag}"])).sum() == 0
    # all-ones weights reduce to plain BP exactly
    ones = g.compact_weights([np.ones((g.E, g.E))] * iters, [np.ones((1, g.n))] * iters, np.ones((g.n, g.E)),
                             np.ones((1, g.n)))
    llr = d["llr_snr1"]
    a = oracle.sp_f32(H, llr, iters, clamp, weights=ones)
    b = oracle.sp_f32(H, llr, iters, clamp)
    assert np.array_equal(a["z"], b["z"])


def test_adc_golden_self_consistent():
    """The ADC fixture's AGC clip is np.std of the stream times the ratio (gen_qdata :118-124)."""
    d = np.load(os.path.join(GOLDEN, "adc_quantizer.npz"))
    rx = d["rx"]
    for i, (b, r) in enumerate(d["agc"]):
        assert np.isclose(d[f"clip_agc{i}"], np.std(rx) * r, rtol=1e-15)


WIFI_SP_FILES = sorted(glob.glob(os.path.join(GOLDEN, "bp_wifi*_sp*.npz")))


@pytest.mark.parametrize("path", WIFI_SP_FILES, ids=lambda p: os.path.basename(p)[3:-4])
def test_oracle_wifi_codes_match_reference(path):
    """(648,1/2), (1296,2/3), (1944,5/6) through the reference module itself (make_golden.py gen_wifi_sp at 5
    iterations, gen_wifi_sp_long at 50 / 20 / 10): the oracle's fp64 p1/z follow the reference's .double() to
    rounding; its fp32 restatement of the reference's operations gives the reference's fp32 hard bits; its
    (D, S) form — the GPU kernels' specification — gives the same bits and satisfies the soft-parity rule
    (tests/softparity.py) that the GPU tests apply."""
    from ldpc_amd.codes import qc_expand
    from softparity import check_p1, check_z, f64_target
    d = np.load(path)
    H = qc_expand(d["base"], int(d["Z"]))
    iters, clamp = int(d["iters"]), float(d["clamp"])
    assert len(WIFI_SP_FILES) == 8
    for snr in d["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        llr = d[f"llr_{tag}"]
        r64 = oracle.sp_f64(H, llr.astype(np.float64), iters, clamp)
        # fp64 vs fp64 in another summation order: rounding, amplified ~1e3x by 50 iterations on decoding failures
        t64 = TOL_P1_F64 if iters <= 10 else 1e-9
        assert np.abs(r64["p1"] - d[f"p1_f64_{tag}"]).max() <= t64
        assert np.abs(r64["z"] - d[f"z_f64_{tag}"]).max() <= 10 * t64 * max(1.0, np.abs(d[f"z_f64_{tag}"]).max())
        ref_bits = np.round(d[f"p1_f32_{tag}"]).astype(np.uint8)
        r32 = oracle.sp_f32(H, llr, iters, clamp)
        assert np.array_equal(r32["bits"], ref_bits)
        rs = oracle.sp_f32(H, llr, iters, clamp, stable=True)
        assert np.array_equal(rs["bits"], ref_bits)
        label = f"oracle-ds {os.path.basename(path)[3:-4]} {tag}"
        p1_t, z_t = f64_target(d, tag, H)
        check_p1(label, rs["p1"], d[f"p1_f32_{tag}"], p1_t, H)
        check_z(label, rs["z"], d[f"z_f32_{tag}"], z_t, H)


def test_ceiling_golden_separates_f32_and_f64_modules():
    """bp_wifi648_12_sp_it50_cl20.npz (clamp 20 > the fp32 ceiling 16.6355): the reference's fp32 and fp64 modules
    differ there by the p-clamp ceiling alone — the oracle's fp64 with the fp64 bound follows .double(); with the
    fp32 bound its z is >= 0.1 away from .double() on ceiling-bound entries and within the reference fp32's own
    near-ceiling quantization of the fp32 module; the (D, S) form follows it to 1e-6 on decoded codewords."""
    from ldpc_amd.codes import qc_expand
    from softparity import CEILING_F32, decoded_rows
    d = np.load(os.path.join(GOLDEN, "bp_wifi648_12_sp_it50_cl20.npz"))
    H = qc_expand(d["base"], int(d["Z"]))
    assert float(d["clamp"]) == 20.0 > CEILING_F32
    llr = d["llr_snr3"]
    t32 = oracle.sp_f64(H, llr.astype(np.float64), 50, 20.0, ceiling="f32")["z"]
    t64 = oracle.sp_f64(H, llr.astype(np.float64), 50, 20.0)["z"]
    assert np.abs(t64 - d["z_f64_snr3"]).max() <= 1e-8 * np.abs(t64).max()
    assert np.abs(t32 - t64).max() > 0.1                     # the two modules' functions differ
    conv = decoded_rows(H, t32)
    assert conv.all()
    rs = oracle.sp_f32(H, llr, 50, 20.0, stable=True)["z"]
    assert (np.abs(rs - t32) / np.maximum(1.0, np.abs(t32))).max() <= 1e-6
    assert (np.abs(d["z_f32_snr3"] - t32) / np.maximum(1.0, np.abs(t32))).max() > 1e-3  # the fp32 module's own


@pytest.mark.parametrize("name", ["bp_wifi648_12_sp_it50_cl20.npz", "bp_wifi1944_56_sp_it50_cl20.npz"])
def test_oracle_f32_bound_f64_pinned_to_reference(name):
    """Above the ceiling the soft target is the REFERENCE's own .double() module with the fp32 module's p-clamp
    bound swapped in at run time (make_golden.py f32_pclamp -> p1_f64b32_* / z_f64b32_*): the oracle's
    sp_f64(ceiling="f32") restates exactly that function — within fp64 rounding of the reference (<= 1e-9 in z over
    50 iterations, decoding failures included); and that target differs from the plain .double() module by the
    ceiling alone (> 0.1 on ceiling-bound entries).  Both clamp-20 files: (648,1/2) BPSK and BASELINE config [2]
    ((1944,5/6), 16-QAM OFDM LLRs)."""
    from ldpc_amd.codes import qc_expand
    d = np.load(os.path.join(GOLDEN, name))
    H = qc_expand(d["base"], int(d["Z"]))
    for snr in d["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        r = oracle.sp_f64(H, d[f"llr_{tag}"].astype(np.float64), int(d["iters"]), float(d["clamp"]), ceiling="f32")
        zb = d[f"z_f64b32_{tag}"]
        assert np.abs(r["z"] - zb).max() <= 1e-9 * max(1.0, np.abs(zb).max())
        assert np.abs(r["p1"] - d[f"p1_f64b32_{tag}"]).max() <= 1e-10
        assert np.abs(zb - d[f"z_f64_{tag}"]).max() > 0.1
        assert np.array_equal(r["bits"], np.round(d[f"p1_f64b32_{tag}"]).astype(np.uint8))


def test_oracle_reference_receiver_chain_golden():
    """e2e_wifi648_qpsk_ofdm.npz: the reference's own receiver chain (QPSK, 32-point OFDM, demodulate_signal)
    into decode_bits(llrs, H, 50, 40, 10) — the oracle's restatement of the reference's fp32 operations decodes
    the decoded rows' LLRs to the same bits (failures included); the tail rows are 0 in the reference's output."""
    from ldpc_amd.codes import qc_expand
    d = np.load(os.path.join(GOLDEN, "e2e_wifi648_qpsk_ofdm.npz"))
    H = qc_expand(d["base"], int(d["Z"]))
    bs, iters = int(d["batch_size"]), int(d["iters"])
    for snr in d["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        llrs, out = d[f"llrs_{tag}"], d[f"out_{tag}"]
        rows = (llrs.shape[0] // bs) * bs
        assert llrs.dtype == np.float64 and out.dtype == np.float64 and not out[rows:].any()
        r = oracle.sp_f32(H, llrs[:rows].astype(np.float32), iters, float(d["clamp"]))
        assert np.array_equal(r["bits"].astype(np.float64), out[:rows])
        assert (out[:rows] != d[f"codeword_{tag}"][:rows]).any()     # the waterfall: failing rows present


def test_oracle_reference_quantized_chain_golden():
    """e2e_quantized.npz: the reference's quantized receiver chain (ADC via gen_qdata, evaluate_quantized.py) into
    decode_bits at clamp 20 — (64,32) with the evaluator's 3-bit ADC at 3 iterations, (648,1/2) with a 5-bit ADC at
    50; LLRs with exact zeros.  Both oracle forms (the reference's fp32 operations and the (D, S) form) give the
    reference's bits on every decoded row, failures included."""
    d = np.load(os.path.join(GOLDEN, "e2e_quantized.npz"))
    for name in ("peg64", "wifi648"):
        H = d[f"H_{name}"].astype(np.int64)
        llrs, out = d[f"llrs_{name}"], d[f"out_{name}"]
        iters, bs, clamp = (int(x) for x in d[f"cfg_{name}"][:3])
        rows = (llrs.shape[0] // bs) * bs
        assert (llrs == 0).any() and not out[rows:].any()
        for stable in (False, True):
            r = oracle.sp_f32(H, llrs[:rows].astype(np.float32), iters, float(clamp), stable=stable)
            assert np.array_equal(r["bits"].astype(np.float64), out[:rows]), (name, stable)


def test_looped_reference_golden_settings():
    """The long-iteration goldens are the drop-in's / BASELINE configs' settings."""
    want = {"wifi648_12": (50, 192), "wifi1296_23": (20, 96), "wifi1944_56": (10, 48)}
    for name, (iters, cws) in want.items():
        d = np.load(os.path.join(GOLDEN, f"bp_{name}_sp_it{iters}.npz"))
        assert int(d["iters"]) == iters and float(d["clamp"]) == 10.0
        assert sum(d[f"llr_snr{s:g}".replace(".", "p")].shape[0] for s in d["snrs"]) == cws
    # BASELINE config [2] at its own settings: (1944,5/6) tanh-SP 50 iterations, the leg's clamp 20, 16-QAM OFDM
    # LLRs from the on-device front end, in the waterfall (6.0 / 6.5 dB: decoded and failing codewords both)
    d = np.load(os.path.join(GOLDEN, "bp_wifi1944_56_sp_it50_cl20.npz"))
    assert int(d["iters"]) == 50 and float(d["clamp"]) == 20.0 and int(d["Z"]) == 81
    assert list(d["snrs"]) == [6.0, 6.5]


def test_ds_form_identities():
    """The (D, S) check rule on hand cases: d = 2 passes the other edge's LLR through, an s = 0 edge zeroes the
    others' messages exactly (the reference's p = 0), a lone edge gets the p-clamp ceiling, the clamp binds."""
    H = np.array([[1, 1, 1, 0], [0, 1, 1, 1]])
    llr = np.array([[2.0, -3.0, 0.0, 1.5], [4.0, 40.0, 1.0, -2.5]], np.float32)
    r = oracle.sp_f32(H, llr, 1, 100.0, trace=True, stable=True)
    x = r["trace"][0]                       # check-order c2v after one iteration, edges (0,0) (0,1) (0,2) (1,1) (1,2) (1,3)
    assert x[0, 0] == 0.0 and x[0, 1] == 0.0  # codeword 0: variable 2 has s = 0 -> edges of check 0 other than it are 0
    f = oracle.sp_f32(H, llr, 1, 100.0, trace=True)["trace"][0]
    assert np.allclose(x, f, rtol=2e-5, atol=1e-6)
    H1 = np.array([[1]])
    r1 = oracle.sp_f32(H1, np.array([[0.5]], np.float32), 1, 100.0, trace=True, stable=True)
    # messages in log2 units (ceiling fp32(log2 16777215) = 24, clamp fp32(clamp * log2 e)), traced times ln 2
    ln2, log2e = np.float32(np.log(2.0)), np.float32(np.log2(np.e))
    assert r1["trace"][0, 0, 0] == np.float32(24.0) * ln2
    assert abs(float(r1["trace"][0, 0, 0]) - np.log(16777215.0)) < 2e-6
    r2 = oracle.sp_f32(H1, np.array([[0.5]], np.float32), 1, 10.0, trace=True, stable=True)
    assert r2["trace"][0, 0, 0] == np.float32(np.float32(10.0) * log2e) * ln2
    assert abs(float(r2["trace"][0, 0, 0]) - 10.0) < 2e-6


def test_degenerate_graph_both_forms():
    """An all-zero row and column of H (the reference accepts any binary H, masking.py:12): both fp32 forms
    decode it (no out-of-range edge access for the empty check) with the same hard bits."""
    H = np.array(np.load(os.path.join(GOLDEN, "peg64_32.npz"))["H"])
    H = np.concatenate([H, np.zeros((1, 64), H.dtype)], axis=0)
    H = np.concatenate([H, np.zeros((33, 1), H.dtype)], axis=1)
    llr = np.random.default_rng(4).normal(2.0, 2.0, size=(100, 65)).astype(np.float32)
    a = oracle.sp_f32(H, llr, 7, 20.0)
    b = oracle.sp_f32(H, llr, 7, 20.0, stable=True)
    assert np.array_equal(a["bits"], b["bits"])
    assert np.allclose(a["z"], b["z"], rtol=1e-4, atol=1e-4)


def test_zero_llr_rows_give_exact_zero_in_both_forms():
    """An all-zero LLR row: the reference's v2c tanh(0) = 0 makes every product 0 and every c2v log(1) = 0, so
    z = 0 exactly and p1 = 0.5 (np.round -> 0).  The (D, S) form: a = 1 for every edge keeps D == S in every
    set, log(S/D) = 0 exactly — the same zeros, not merely small values."""
    H = np.array(np.load(os.path.join(GOLDEN, "peg64_32.npz"))["H"])
    llr = np.zeros((3, 64), np.float32)
    llr[1, ::2] = 2.5                      # half zeros: the zero variables' checks still see exact zeros
    for stable in (False, True):
        r = oracle.sp_f32(H, llr, 10, 10.0, stable=stable)
        assert np.all(r["z"][0] == 0.0) and np.all(r["p1"][0] == 0.5) and not r["bits"][0].any()
    a = oracle.sp_f32(H, llr, 10, 10.0)
    b = oracle.sp_f32(H, llr, 10, 10.0, stable=True)
    assert np.array_equal(a["bits"], b["bits"])
    assert np.allclose(a["z"], b["z"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("code", ["peg64_32", "wifi648_12"])
def test_oracle_clustered_zero_llrs_golden(code):
    """Clustered exact-zero LLRs through the reference (tests/golden/bp_zeros.npz: 2-3 zeros of both signs in a
    third of the checks, 1/2/3/5 iterations, clamp 10 and 20): the oracle's (D, S) form gives exact zeros where
    the reference does (an edge whose exclusive set holds an a == 1 edge outputs +-0, cn_stable_f32) and the
    reference's fp32 bits outside the rounding band (softparity.check_zeros_golden).  Before the rule the fma
    join left ulp-sized outputs there and flipped 1-6 hard decisions."""
    from softparity import check_zeros_golden
    from ldpc_amd.codes import get_code
    d = np.load(os.path.join(GOLDEN, "bp_zeros.npz"))
    H = np.asarray(get_code(code)[0])
    x = d[f"{code}_llr"]
    for it in (1, 2, 3, 5):
        for cl in (10, 20):
            r = oracle.sp_f32(H, x, it, float(cl), stable=True)
            check_zeros_golden(f"oracle-ds zeros {code}", r["bits"], r["z"], d, f"{code}_it{it}_cl{cl}")
