"""Soft-output parity against the reference's float64 output (north_star: soft outputs within 1e-5).

The reference's own fp32 forward is not a fixed target: near |p| -> 1 its fp32 `log((1+p)/(1-p))`
(`bp/bp_cv.py:44-50`) is ill-conditioned, so torch-fp32 and any other fp32 evaluation (ours: the same
operations with the GPU's tanhf/logf/expf) drift apart from each other and from fp64 on a few entries.
The rule used by every soft-parity test:

* **p1** (`BeliefPropagation.forward`'s output, `bp/bp.py:51`): on every entry where the reference's
  fp32 p1 is within 1e-5 of the reference's fp64 p1 ("well-conditioned"), ours must be within 1e-5 of
  the reference's fp64 p1.  The excluded (ill-conditioned) entries are counted and reported.
* **z** (the final VC output, `bp_vc.py:16-27` with `mask_v_final`; an LLR of magnitude up to ~50,
  where one fp32 ulp is 4e-6): ours must stay inside the reference's own fp32 error envelope,
  |z - z64| <= Z_ENVELOPE * max(|z32 - z64|, 1e-5 * max(1, |z64|)), i.e. no worse than a small factor of
  what the reference itself achieves in fp32, and 1e-5-relative where the reference's fp32 is.

Each check appends its measured maxima to $LDPC_PARITY_LOG (JSON lines) when that is set; the GPU
scripts collect them into profiles/.
"""
import json
import os

import numpy as np

TOL = 1e-5
Z_ENVELOPE = 3.0  # measured maximum ratio 2.70 (GPU and C oracle alike; profiles/r02/soft_parity.jsonl)


def _log(rec):
    path = os.environ.get("LDPC_PARITY_LOG")
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def check_p1(label, got, ref32, ref64, tol=TOL):
    """got/ref32/ref64: p1 arrays of one shape.  Returns the record (also logged)."""
    got = np.asarray(got, np.float64)
    ref32 = np.asarray(ref32, np.float64)
    ref64 = np.asarray(ref64, np.float64)
    ok = np.abs(ref32 - ref64) <= tol
    err = np.abs(got - ref64)
    rec = {"label": label, "kind": "p1", "entries": int(err.size), "excluded_ill_conditioned": int((~ok).sum()),
           "max_abs_vs_ref_f64_on_well_conditioned": float(err[ok].max()) if ok.any() else 0.0,
           "max_abs_vs_ref_f64_all": float(err.max()) if err.size else 0.0,
           "ref_f32_vs_ref_f64_max": float(np.abs(ref32 - ref64).max()) if err.size else 0.0,
           "tol": tol}
    _log(rec)
    bad = int((err[ok] > tol).sum())
    assert bad == 0, f"{label}: {bad} well-conditioned p1 entries off by > {tol}: {rec}"
    return rec


def check_z(label, got, z32, z64, envelope=Z_ENVELOPE):
    got = np.asarray(got, np.float64)
    z32 = np.asarray(z32, np.float64)
    z64 = np.asarray(z64, np.float64)
    scale = np.maximum(1.0, np.abs(z64))
    ref_err = np.abs(z32 - z64)
    err = np.abs(got - z64)
    ok = ref_err <= TOL * scale
    ratio = err / np.maximum(ref_err, TOL * scale)
    rec = {"label": label, "kind": "z", "entries": int(err.size), "ref_f32_outside_1e-5_rel": int((~ok).sum()),
           "max_rel_vs_ref_f64_where_ref_f32_within_1e-5": float((err / scale)[ok].max()) if ok.any() else 0.0,
           "entries_rel_gt_1e-5_where_ref_f32_within": int(((err / scale)[ok] > TOL).sum()),
           "max_abs_vs_ref_f64": float(err.max()), "ref_f32_max_abs_vs_ref_f64": float(ref_err.max()),
           "max_envelope_ratio": float(ratio.max()), "envelope": envelope}
    _log(rec)
    assert rec["max_envelope_ratio"] <= envelope, f"{label}: z outside the reference's fp32 envelope: {rec}"
    return rec
