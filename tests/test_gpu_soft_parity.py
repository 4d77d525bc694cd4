"""Soft-output parity of the HIP tanh-SP decoder against the REFERENCE's float64 output
(north_star: within 1e-5 on soft outputs; rule in tests/softparity.py).

Goldens were produced by the reference itself (tests/golden/make_golden.py):
* bp_peg64_snr*.npz: the (64,32) PEG code, Eb/N0 {0,2,4} x (iters, clamp) {(3,20),(5,10),(10,10),(10,100),(50,10)};
* bp_<802.11n code>_sp.npz: (648,1/2) 128 codewords, (1296,2/3) and (1944,5/6) 32 codewords each, 5 iterations,
  clamp 10, p1 and z in fp32 and fp64 (`bp/bp.py:43-51`, `bp_vc.py:16-27`, `bp_cv.py:22-50`);
* bp_<802.11n code>_sp_it<k>.npz: the same at the iteration counts the drop-in and the BASELINE configs run —
  (648,1/2) 50 iterations x 192 codewords, (1296,2/3) 20 x 96, (1944,5/6) 10 x 48, clamp 10;
* bp_wifi648_12_sp_it50_cl20.npz: (648,1/2) 50 iterations, clamp 20 — above the p-clamp ceiling, where the z target
  is the fp32 module's function in fp64 (softparity.f64_target);
* bp_wifi1944_56_sp_it50_cl20.npz: BASELINE config [2] at its own settings — (1944,5/6), 50 iterations, clamp 20,
  16-QAM OFDM LLRs from the on-device front end, 16 codewords at 6.0 and 6.5 dB.
Both kernel families run every file: the register/sliced QC kernels ("auto") and the generic CSR kernels.
Hard decisions must equal the reference's fp32 hard decisions exactly.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN
from softparity import check_p1, check_z, f64_target

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd.codes import qc_expand  # noqa: E402

PEG_FILES = sorted(glob.glob(os.path.join(GOLDEN, "bp_peg64_snr*.npz")))
WIFI_FILES = sorted(glob.glob(os.path.join(GOLDEN, "bp_wifi*_sp*.npz")))


def _name(p):
    return os.path.basename(p)[3:-4]


@pytest.mark.parametrize("path", PEG_FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_peg64_p1_vs_reference_f64(path):
    d = np.load(path)
    dec = ldpc_amd.get_decoder(d["H"])
    r = dec.decode(torch.from_numpy(d["llr"]).cuda(), int(d["iters"]), algo="tanh", clamp=float(d["clamp"]), soft="p1")
    p1 = r["soft"].cpu().numpy()
    assert np.array_equal(r["bits"].cpu().numpy(), d["bits_f32"])
    check_p1(os.path.basename(path)[:-4], p1, d["p1_f32"], d["p1_f64"], d["H"])


@pytest.mark.parametrize("path", WIFI_FILES, ids=_name)
@pytest.mark.parametrize("path_kind", ["auto", "generic"])
def test_wifi_p1_and_z_vs_reference_f64(path, path_kind):
    d = np.load(path)
    H = qc_expand(d["base"], int(d["Z"]))
    dec = ldpc_amd.get_decoder(H)
    if path_kind == "auto":
        assert dec.qc_z == int(d["Z"])  # the QC kernel family is the one under test
    iters, clamp = int(d["iters"]), float(d["clamp"])
    name = _name(path)
    for snr in d["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        x = torch.from_numpy(d[f"llr_{tag}"]).cuda()
        fg = path_kind == "generic"
        rp = dec.decode(x, iters, algo="tanh", clamp=clamp, soft="p1", force_generic=fg)
        rz = dec.decode(x, iters, algo="tanh", clamp=clamp, soft="z", force_generic=fg)
        ref_bits = np.round(d[f"p1_f32_{tag}"]).astype(np.uint8)
        assert np.array_equal(rp["bits"].cpu().numpy(), ref_bits)
        assert np.array_equal(rz["bits"].cpu().numpy(), ref_bits)
        label = f"{name} {tag} {path_kind}"
        p1_t, z_t = f64_target(d, tag, H)
        check_p1(label, rp["soft"].cpu().numpy(), d[f"p1_f32_{tag}"], p1_t, H)
        check_z(label, rz["soft"].cpu().numpy(), d[f"z_f32_{tag}"], z_t, H)


@pytest.mark.parametrize("path", WIFI_FILES, ids=_name)
def test_wifi_f64_vs_reference_f64(path):
    """precision='f64' (generic kernels) against the reference's .double() module."""
    d = np.load(path)
    H = qc_expand(d["base"], int(d["Z"]))
    dec = ldpc_amd.get_decoder(H)
    for snr in d["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        llr = d[f"llr_{tag}"].astype(np.float64)
        r = dec.decode(llr, int(d["iters"]), algo="tanh", clamp=float(d["clamp"]), soft="z", precision="f64")
        tol = 1e-10 if int(d["iters"]) <= 10 else 1e-8  # fp64 rounding, amplified on decoding failures at 50 it
        assert np.abs(r["soft"] - d[f"z_f64_{tag}"]).max() <= tol * max(1.0, np.abs(d[f"z_f64_{tag}"]).max())
        assert np.array_equal(r["bits"], np.round(d[f"p1_f64_{tag}"]).astype(np.uint8))
