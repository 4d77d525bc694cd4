"""Weighted BP on the GPU: the reference module with trained (non-unit) VC weights (bp_vc.py:16-27),
against the reference's own outputs (tests/golden/bp_weighted_peg64.npz) and the weighted oracle."""
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
from ldpc_amd.api import get_decoder  # noqa: E402
from ldpc_amd.codes import Graph, get_code  # noqa: E402

D = np.load(os.path.join(GOLDEN, "bp_weighted_peg64.npz"))
ITERS, CLAMP = int(D["iters"]), float(D["clamp"])


def _state_dict():
    sd = {}
    for i in range(ITERS):
        sd[f"layers.{i}.0.input_weight"] = torch.from_numpy(D[f"input_weight{i}"])
        sd[f"layers.{i}.0.llr_weight"] = torch.from_numpy(D[f"llr_weight{i}"])
    sd["final_layer.0.input_weight"] = torch.from_numpy(D["final_input_weight"])
    sd["final_layer.0.llr_weight"] = torch.from_numpy(D["final_llr_weight"])
    return sd


@pytest.mark.parametrize("tag", ["snr1", "snr3"])
def test_module_weighted_matches_reference(tag):
    m = ldpc_amd.BeliefPropagation(D["H"], ITERS).load_reference_state_dict(_state_dict())
    llr = torch.from_numpy(D[f"llr_{tag}"]).cuda()
    x = torch.zeros(llr.shape[0], m.layer_size(), device="cuda")
    p1 = m(x, llr, CLAMP).cpu().numpy()
    ref = D[f"p1_f32_{tag}"]
    check_p1(f"weighted peg64 {tag}", p1, ref, D[f"p1_f64_{tag}"], D["H"])
    assert np.array_equal(np.round(p1), np.round(ref))
    p64 = m.double()(x.double(), llr.double(), CLAMP).cpu().numpy()
    assert np.abs(p64 - D[f"p1_f64_{tag}"]).max() < 1e-10


def _random_weights(g, iters, rng):
    return dict(vn=rng.uniform(0.3, 1.7, (iters, int(g.weight_offsets()[-1]))),
                llr=rng.uniform(0.5, 1.5, (iters, g.n)), fin=rng.uniform(0.5, 1.5, g.E),
                fin_llr=rng.uniform(0.5, 1.5, g.n))


@pytest.mark.parametrize("code", ["wifi648_12", "wifi1296_23"])
def test_weighted_vs_oracle(code):
    H, _ = get_code(code)
    g = Graph.from_H(H)
    rng = np.random.default_rng(7)
    iters = 8
    w = _random_weights(g, iters, rng)
    llr = (rng.standard_normal((300, g.n)) * 2.5 + 1.5).astype(np.float32)
    d = get_decoder(H)
    r = d.decode(torch.from_numpy(llr).cuda(), iters, algo="tanh", clamp=10.0, soft="z", weights=w)
    o = oracle.sp_f32(g, llr, iters, 10.0, weights={k: v.astype(np.float32) for k, v in w.items()}, stable=True)
    z = r["soft"].cpu().numpy()
    rel = float((np.abs(z.astype(np.float64) - o["z"]) / np.maximum(1.0, np.abs(o["z"]))).max())
    _log({"label": f"weighted_vs_oracle {code}", "kind": "z_rel_vs_oracle", "max": rel})
    assert rel < 5e-6   # measured 7.2e-7 (profiles/r02/soft_parity.jsonl)
    close = np.abs(o["z"]) > 1e-3
    assert np.array_equal(r["bits"].cpu().numpy()[close], o["bits"][close])
    r64 = d.decode(llr.astype(np.float64), iters, algo="tanh", clamp=10.0, soft="z", precision="f64", weights=w)
    o64 = oracle.sp_f64(g, llr.astype(np.float64), iters, 10.0, weights=w)
    assert np.abs(r64["soft"] - o64["z"]).max() < 1e-9


def test_ones_weights_equal_plain_bp_bitwise():
    H, _ = get_code("wifi648_12")
    g = Graph.from_H(H)
    rng = np.random.default_rng(3)
    llr = torch.from_numpy((rng.standard_normal((257, g.n)) * 2 + 1).astype(np.float32)).cuda()
    d = get_decoder(H)
    ones = dict(vn=np.ones((6, int(g.weight_offsets()[-1]))), llr=np.ones((6, g.n)), fin=np.ones(g.E),
                fin_llr=np.ones(g.n))
    a = d.decode(llr, 6, algo="tanh", soft="z", weights=ones)["soft"]
    b = d.decode(llr, 6, algo="tanh", soft="z", force_generic=True)["soft"]
    assert torch.equal(a, b)
    c = d.decode(llr, 6, algo="tanh", soft="z", weights={})["soft"]   # all-None = ones
    assert torch.equal(a, c)


def test_weighted_errors():
    H, _ = get_code("wifi648_12")
    d = get_decoder(H)
    llr = torch.zeros((4, 648), device="cuda")
    with pytest.raises(_abi.LdpcError):
        d.decode(llr, 3, algo="minsum", weights={})
    with pytest.raises(_abi.LdpcError):
        d.decode(llr, 3, algo="tanh", early_stop=True, weights={})
    with pytest.raises(ValueError):
        d.decode(llr, 3, algo="tanh", weights=dict(llr=np.ones((2, 648))))
