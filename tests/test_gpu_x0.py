"""BeliefPropagation.forward with NON-ZERO initial messages x (pytorch/bp/bp.py:43-47): the reference's first
layer consumes x like any later layer's c2v.  Pinned to reference-run goldens (tests/golden/bp_x0.npz,
make_golden.py gen_x0): p1 within 1e-5 of the reference's fp64 on well-conditioned entries (softparity.py),
fp64 within 1e-10, hard decisions identical to the reference's fp32 np.round(p1)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from softparity import check_p1

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd.codes import get_code  # noqa: E402

CASES = [("peg64_32", 0), ("peg64_32", 1), ("peg64_32", 5), ("wifi648_12", 3)]


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLDEN, "bp_x0.npz"))


@pytest.mark.parametrize("name,iters", CASES)
@pytest.mark.parametrize("where", ["cuda", "cpu"])
def test_forward_with_initial_messages(gold, name, iters, where):
    H = np.asarray(get_code(name)[0])
    llr = torch.from_numpy(gold[f"{name}_llr"]).to(where)
    x = torch.from_numpy(gold[f"{name}_x"]).to(where)
    m = ldpc_amd.BeliefPropagation(H, iters).eval()
    assert m.layer_size() == x.shape[1]
    p1 = m(x, llr, 10.0)
    assert p1.device.type == where
    p1 = p1.cpu().numpy()
    r32, r64 = gold[f"{name}_it{iters}_p1_f32"], gold[f"{name}_it{iters}_p1_f64"]
    check_p1(f"x0 {name} it{iters} {where}", p1, r32, r64, H)
    assert np.array_equal(np.round(p1), np.round(r32))
    if where == "cuda":
        p64 = m.double()(x.double(), llr.double(), 10.0).cpu().numpy()
        assert np.abs(p64 - r64).max() <= 1e-10


def test_zero_x_takes_the_plain_path(gold):
    """x = 0 is what every reference caller passes; it must equal decoding without x0 bit for bit."""
    H = np.asarray(get_code("wifi648_12")[0])
    llr = torch.from_numpy(gold["wifi648_12_llr"]).cuda()
    m = ldpc_amd.BeliefPropagation(H, 3).eval()
    a = m(torch.zeros(llr.shape[0], m.layer_size(), device="cuda"), llr, 10.0)
    dec = ldpc_amd.get_decoder(H)
    b = dec.decode(llr, 3, algo="tanh", clamp=10.0, soft="p1", want_bits=False,
                   x0=torch.zeros(llr.shape[0], m.layer_size(), device="cuda"))["soft"]
    assert torch.equal(a, b)
