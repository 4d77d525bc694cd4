"""Decodes captured into a CUDA (HIP) graph and replayed on new LLRs equal the eager decodes bit for bit: the IRA
path with several Infinity-Cache chunks round-robin over its own streams (fixed count and early stop, whose
convergence words are cleared by a memset inside the graph), the packed 5-bit kernel with early stop and the
headline min-sum kernel.  (The tanh-SP zero pass: tests/test_gpu_zero_pass.py.)  A caller that replays a whole
BER point as one graph launch needs every decode path capturable: no host synchronisation, allocation or
stream creation inside a decode once the decoder is warm."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd.codes import Encoder, IRAEncoder, get_code  # noqa: E402


def _llr(H, enc, B, ebn0, seed):
    rng = np.random.default_rng(seed)
    cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
    sigma = np.sqrt(1.0 / (10 ** (ebn0 / 10)))
    return (-2.0 * ((1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)) / sigma**2).astype(np.float32)


CASES = [
    ("dvbs2_12", 11, dict(algo="minsum", clamp=20.0)),
    ("dvbs2_12", 11, dict(algo="minsum", clamp=20.0, early_stop=True)),
    ("wifi1296_23", 600, dict(algo="qminsum", qstep=1.0, early_stop=True)),
    ("wifi648_12", 1000, dict(algo="minsum", clamp=20.0)),
]


@pytest.mark.parametrize("name,B,kw", CASES, ids=["ira", "ira-es", "packed-es", "minsum-ph"])
def test_graph_replay_equals_eager(name, B, kw, monkeypatch):
    monkeypatch.setenv("LDPC_IRA_BUDGET_MB", "3")      # several chunks
    H, _ = get_code(name)
    enc = IRAEncoder(H) if name.startswith("dvbs2") else Encoder(H)
    dec = ldpc_amd.get_decoder(H)
    iters = 14
    kw = dict(kw, soft="z", want_iters=True)
    xt = torch.from_numpy(_llr(H, enc, B, 1.8, seed=1)).cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):  # warm: workspace, device tables, streams and events exist before capture
            dec.decode(xt, iters, **kw)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = dec.decode(xt, iters, **kw)
    for seed, ebn0 in ((2, 2.6), (3, 1.2)):
        x1 = _llr(H, enc, B, ebn0, seed)
        xt.copy_(torch.from_numpy(x1).cuda())
        graph.replay()
        torch.cuda.synchronize()
        ref = dec.decode(torch.from_numpy(x1).cuda(), iters, **kw)
        torch.cuda.synchronize()
        assert torch.equal(out["bits"], ref["bits"]), seed
        assert torch.equal(out["soft"].view(torch.int32), ref["soft"].view(torch.int32)), seed
        assert torch.equal(out["iters_used"], ref["iters_used"]), seed
