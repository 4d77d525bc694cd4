"""Soft-output parity against the reference's float64 output (north_star: soft outputs within 1e-5).

The decoder's fp32 tanh-SP evaluates the reference's check rule (`bp/bp_cv.py:38-50`) in the (D, S) form
(`ldpc-sims_amd/csrc/common.h`, `oracle/ldpc_oracle.c` cn_stable_f32): sums of positive terms instead of the
reference's `log((1+p)/(1-p))`, whose `1-p` cancels near |p| -> 1 (one fp32 ulp of tanh there is a 1e-4..1e-3
error in the log).  So the target is the reference's fp64 output, and the rules are:

* **p1** (`BeliefPropagation.forward`'s output, `bp/bp.py:51`; absolute) and
* **z** (the final VC output, `bp_vc.py:16-27` with `mask_v_final`; an LLR up to ~50; relative to max(1, |z|)):
  - on every codeword the reference DECODES (its fp64 hard decision satisfies every check — H b = 0):
    |z - z64| <= 1e-5 * max(1, |z64|) on **every** entry, no exclusions;
  - on decoding failures (oscillating / non-convergent codewords) BP's iteration map amplifies any fp32
    rounding (fp64 VN sums change nothing there: DESIGN.md §4), so fp32 cannot follow fp64 to 1e-5 after
    tens of iterations — the reference's own fp32 is off by up to 2e-3 there.  Asserted, per golden set:
    (i) the maximum is within max(1e-5, the reference's own fp32 error on the failing codewords of the set);
    (ii) the maximum and (iii) the number of entries where the reference's fp32 meets 1e-5 and ours does not
    are at most their MEASURED values (FAILURE_BOUNDS: the GPU kernels — register, sliced and generic CSR
    give bitwise-equal z — and the C oracle's (D, S) form, each measured; a set not listed must have none).
    A change of the fp32 arithmetic that moves any of them fails here and must re-measure (DESIGN §4 holds
    the trace of where the failing codewords leave the reference's fp32).

A caller's clamp above the fp32 module's p-clamp ceiling log(16777215) = 16.6355 (bp_cv.py:44-47 with the bound
1-1e-7 rounded to fp32) lets messages reach that ceiling, which the .double() module puts at log(19999999) =
16.8112 instead: the fp32 and fp64 modules then compute different functions.  The decoder is an fp32 drop-in, so
for such files the p1 and z targets are `f64_target`: the REFERENCE's own .double() module run with the fp32 module's
bound swapped in at run time (tests/golden/make_golden.py f32_pclamp: p1_f64b32_* / z_f64b32_*; the oracle's
sp_f64(ceiling="f32") follows it to 1e-9, tests/test_oracle_golden.py), equal to the plain .double() module wherever
no message reaches either ceiling.

Each check appends its measured maxima to $LDPC_PARITY_LOG (JSON lines) when that is set; the GPU
scripts collect them into profiles/.
"""
import json
import os

import numpy as np

TOL = 1e-5
# (kind, golden set, implementation) -> (entries where the reference's fp32 is within 1e-5 and ours is not, the
# maximum error on decoding failures): measured with the fma join (common.h DS_JOIN_FMA; GPU: the -m gpu suite
# under LDPC_PARITY_MEASURE=1, every kernel family, profiles/r04/failure_bounds/; oracle: the CPU suite), collected
# by scripts/failure_bounds.py, the maxima rounded up in the third digit.  Unlisted sets: count 0.
FAILURE_BOUNDS = {
    ("z", "wifi648_12_sp_it50 snr1", "gpu"): (281, 1.94e-4),
    ("p1", "wifi648_12_sp_it50 snr1", "gpu"): (24, 4.45e-5),
    ("z", "wifi648_12_sp_it50 snr2", "gpu"): (19, 3.84e-4),
    ("p1", "wifi648_12_sp_it50 snr2", "gpu"): (21, 8.02e-5),
    ("z", "wifi648_12_sp_it50_cl20 snr2", "gpu"): (17, 3.63e-4),
    ("p1", "wifi648_12_sp_it50_cl20 snr2", "gpu"): (16, 8.13e-5),
    ("z", "wifi1296_23_sp_it20 snr2", "gpu"): (1, 1.12e-5),
    ("z", "wifi1944_56_sp_it50_cl20 snr6", "gpu"): (12, 3.68e-5),  # config [2]: 13 of 16 fail at 6.0 dB
    ("z", "wifi648_12_sp_it50 snr1", "oracle"): (97, 6.67e-5),
    ("p1", "wifi648_12_sp_it50 snr1", "oracle"): (2, 1.53e-5),
    ("z", "wifi648_12_sp_it50 snr2", "oracle"): (22, 8.85e-4),
    ("p1", "wifi648_12_sp_it50 snr2", "oracle"): (29, 2.21e-4),
    ("z", "wifi648_12_sp_it50_cl20 snr2", "oracle"): (18, 6.87e-4),
    ("p1", "wifi648_12_sp_it50_cl20 snr2", "oracle"): (27, 1.71e-4),
}


def _bounds(kind, label):
    """FAILURE_BOUNDS entry of a check label ('<set> <tag> auto|generic' for the GPU, 'oracle-ds <set> <tag>')."""
    parts = label.split()
    impl = "oracle" if parts[0] == "oracle-ds" else "gpu"
    key = " ".join(parts[1:3]) if impl == "oracle" else " ".join(parts[:2])
    return FAILURE_BOUNDS.get((kind, key, impl))
CEILING_F32 = float(np.log(np.float64(16777215.0)))  # log((1+p)/(1-p)) at p = (float)(1-1e-7)


def f64_target(d, tag, H):
    """(p1, z): the fp64 targets of golden file `d` at Eb/N0 tag `tag` (see the module docstring)."""
    clamp = float(d["clamp"])
    if clamp <= CEILING_F32:
        return d[f"p1_f64_{tag}"], d[f"z_f64_{tag}"]
    return d[f"p1_f64b32_{tag}"], d[f"z_f64b32_{tag}"]   # the reference's fp64 module with the fp32 bound


def _log(rec):
    path = os.environ.get("LDPC_PARITY_LOG")
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def check_p1(label, got, ref32, ref64, H, tol=TOL):
    """got/ref32/ref64: p1 arrays of one shape; H the code.  On codewords the reference decodes (its fp64
    decision p1 > 0.5 satisfies H) every entry within `tol` of the fp64 p1; on decoding failures within
    max(tol, the reference's own fp32 error there).  Returns the record (also logged)."""
    got = np.asarray(got, np.float64)
    ref32 = np.asarray(ref32, np.float64)
    ref64 = np.asarray(ref64, np.float64)
    err = np.abs(got - ref64)
    ref_err = np.abs(ref32 - ref64)
    conv = decoded_rows(H, 0.5 - ref64)  # p1 > 0.5 <=> bit 1 <=> z < 0
    fail_env = float(ref_err[~conv].max()) if (~conv).any() else 0.0
    rec = {"label": label, "kind": "p1", "entries": int(err.size), "decoded_codewords": int(conv.sum()),
           "codewords": int(err.shape[0]),
           "max_abs_on_decoded": float(err[conv].max()) if conv.any() else 0.0,
           "ref_f32_max_abs_on_decoded": float(ref_err[conv].max()) if conv.any() else 0.0,
           "max_abs_on_failures": float(err[~conv].max()) if (~conv).any() else 0.0,
           "ref_f32_max_abs_on_failures": fail_env,
           "failures_entries_gt_tol_where_ref_f32_within": int(((err > tol) & (ref_err <= tol) & ~conv[:, None]).sum()),
           "tol": tol}
    _log(rec)
    bad = int((err[conv] > tol).sum())
    assert bad == 0, f"{label}: {bad} p1 entries of decoded codewords off by > {tol}: {rec}"
    _check_failures(rec, "p1", rec["max_abs_on_failures"], fail_env, "failures_entries_gt_tol_where_ref_f32_within", tol)
    return rec


def decoded_rows(H, z64):
    """Codewords whose fp64 reference hard decision (z < 0 <=> bit 1) satisfies every check of H."""
    b = (np.asarray(z64) < 0).astype(np.int64)
    return ~((b @ np.asarray(H, np.int64).T) % 2).any(axis=1)


def check_z(label, got, z32, z64, H):
    got = np.asarray(got, np.float64)
    z32 = np.asarray(z32, np.float64)
    z64 = np.asarray(z64, np.float64)
    scale = np.maximum(1.0, np.abs(z64))
    err = np.abs(got - z64) / scale
    ref_err = np.abs(z32 - z64) / scale
    conv = decoded_rows(H, z64)
    fail_env = float(ref_err[~conv].max()) if (~conv).any() else 0.0
    ref_ok = ref_err <= TOL
    rec = {"label": label, "kind": "z", "entries": int(err.size), "codewords": int(err.shape[0]),
           "decoded_codewords": int(conv.sum()),
           "max_rel_on_decoded": float(err[conv].max()) if conv.any() else 0.0,
           "ref_f32_max_rel_on_decoded": float(ref_err[conv].max()) if conv.any() else 0.0,
           "max_rel_on_failures": float(err[~conv].max()) if (~conv).any() else 0.0,
           "ref_f32_max_rel_on_failures": fail_env,
           "failures_entries_rel_gt_1e-5_where_ref_f32_within": int(((err > TOL) & ref_ok & ~conv[:, None]).sum()),
           "tol": TOL}
    _log(rec)
    bad = int((err[conv] > TOL).sum())
    assert bad == 0, f"{label}: {bad} z entries of decoded codewords off by > {TOL} relative: {rec}"
    _check_failures(rec, "z", rec["max_rel_on_failures"], fail_env, "failures_entries_rel_gt_1e-5_where_ref_f32_within",
                    TOL)
    return rec


def _check_failures(rec, kind, got_max, ref_env, count_key, tol):
    """The decoding-failure rules (module docstring): (i) within max(tol, the reference's own fp32 error),
    (ii) + (iii) the maximum and the count at most their measured values."""
    label = rec["label"]
    assert got_max <= max(tol, ref_env), f"{label}: {kind} on decoding failures outside max({tol}, the reference's " \
                                         f"own fp32 error there): {rec}"
    if os.environ.get("LDPC_PARITY_MEASURE"):  # re-measuring FAILURE_BOUNDS (scripts/failure_bounds.py): (i) only
        return
    count_m, max_m = _bounds(kind, label) or (0, max(tol, ref_env))
    assert rec[count_key] <= count_m, f"{label}: {rec[count_key]} {kind} entries where the reference's fp32 meets " \
                                      f"{tol} and ours does not (measured bound {count_m}): {rec}"
    assert got_max <= max_m, f"{label}: {kind} maximum on decoding failures {got_max:.3e} above the measured " \
                             f"{max_m:.3e}: {rec}"


# Clustered exact-zero LLRs (tests/golden/bp_zeros.npz): hard decisions within this band of the
# reference's fp64 z are decided by rounding — the reference's own fp32 and fp64 modules disagree there (up to 302
# of 16 x 648 bits at 5 iterations) — so the bits are held to the reference's fp32 outside it, and inside it to
# at most as many disagreements as the reference's fp32 has with its own fp64.
ZERO_BAND = 1e-6


def check_zeros_golden(label, bits, z, d, tag):
    """bits / z of one bp_zeros.npz case (`tag` = '<code>_it<k>_cl<c>') against the reference: wherever the
    reference's fp64 z is exactly 0, |z| <= 2^-23 (exactly 0 but where messages cancel to the last bit in the
    reference's arithmetic: 1 of 1,013 at 5 iterations — the s = +-0 rule, cn_ds_row FIX / oracle cn_stable_f32,
    makes the rest exact; before it the fma join left up to 2.4e-7 and flipped bits); bits equal to
    the reference's fp32 outside ZERO_BAND; inside it no more disagreements than the reference's fp32 vs fp64;
    z within 1e-5 relative (scale max(1, |z|)) of the fp64 z."""
    z64 = d[f"{tag}_z_f64"]
    b32 = np.round(d[f"{tag}_p1_f32"]).astype(np.uint8)
    b64 = np.round(d[f"{tag}_p1_f64"]).astype(np.uint8)
    band = np.abs(z64) < ZERO_BAND
    zero = z64 == 0
    rec = {"label": label, "kind": "zeros", "tag": tag, "exact_zero_ref": int(zero.sum()),
           "exact_zero_ours": int((z[zero] == 0).sum()), "max_abs_z_at_ref_zero": float(np.abs(z[zero]).max()),
           "band": int(band.sum()),
           "mismatch_outside_band": int(((bits != b32) & ~band).sum()),
           "mismatch_in_band": int(((bits != b32) & band).sum()),
           "ref32_vs_ref64_in_band": int(((b32 != b64) & band).sum()),
           "z_rel_max": float((np.abs(z - z64) / np.maximum(1.0, np.abs(z64))).max())}
    _log(rec)
    assert rec["max_abs_z_at_ref_zero"] <= 2.0 ** -23, rec
    assert rec["exact_zero_ours"] >= rec["exact_zero_ref"] - 2, rec
    assert rec["mismatch_outside_band"] == 0, rec
    assert rec["mismatch_in_band"] <= rec["ref32_vs_ref64_in_band"], rec
    assert rec["z_rel_max"] <= TOL, rec
    return rec
