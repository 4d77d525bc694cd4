"""The tanh-SP register kernels' a == 1 pass at scale (csrc/qc.hip k_sp_zero_scan / qc_sp_fork): the scan lists
the waves / units whose LLRs hold an exact zero, the rule's pass walks that list on a second stream beside the
plain pass.  Every unit listed (more than the second pass's grid, so its workgroups walk several entries), none
listed, a ragged batch; graph capture of the forked decode.  Bitwise against the generic kernels, which apply
the rule everywhere."""
import numpy as np
import pytest

from ldpc_amd.codes import Encoder, get_code

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402


def _llr(H, B, snr_db, seed):
    rng = np.random.default_rng(seed)
    enc = Encoder(H)
    rate = enc.k / H.shape[1]
    cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
    sigma = np.sqrt(1.0 / (2 * rate * 10 ** (snr_db / 10)))
    y = (1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)
    return (-2.0 * y / sigma**2).astype(np.float32)


def _same(a, g):
    return (torch.equal(a["bits"], g["bits"]) and torch.equal(a["soft"].view(torch.int32), g["soft"].view(torch.int32))
            and (a["iters_used"] is None or torch.equal(a["iters_used"], g["iters_used"])))


# (code, B): B such that every wave / unit listed exceeds the second pass's grid (1,280 workgroups: 5,120 waves
# of the stored kernels, 1,280 units of the sliced ones), odd B for a ragged last wave / unit
@pytest.mark.parametrize("code,B", [("wifi648_12", 10241), ("wifi1296_23", 5123), ("wifi1944_56", 2601)])
@pytest.mark.parametrize("early", [False, True])
def test_every_unit_listed(code, B, early):
    H = np.asarray(get_code(code)[0])
    dec = ldpc_amd.get_decoder(H)
    x = _llr(H, B, 3.0, seed=B)
    x[:, 5] = 0.0                                      # one erasure per codeword: every unit listed
    x[1::7, 40:44] = -0.0
    xt = torch.from_numpy(x).cuda()
    kw = dict(algo="tanh", clamp=20.0, soft="z", early_stop=early, want_iters=True)
    a = dec.decode(xt, 12, **kw)
    g = dec.decode(xt, 12, force_generic=True, **kw)
    assert _same(a, g)


@pytest.mark.parametrize("code", ["wifi648_12", "wifi1944_56"])
def test_none_and_one_listed(code):
    """No zero at all (the second pass walks an empty list), then one zero in the batch's last codeword."""
    H = np.asarray(get_code(code)[0])
    dec = ldpc_amd.get_decoder(H)
    x = _llr(H, 777, 3.0, seed=3)
    x[x == 0.0] = 1e-3
    kw = dict(algo="tanh", clamp=20.0, soft="z", want_iters=True)
    for case in ("none", "last"):
        if case == "last":
            x[-1, 100] = 0.0
        xt = torch.from_numpy(x).cuda()
        assert _same(dec.decode(xt, 15, **kw), dec.decode(xt, 15, force_generic=True, **kw)), case


@pytest.mark.parametrize("code", ["wifi648_12", "wifi1944_56"])
def test_graph_capture_of_forked_decode(code):
    """The forked decode (scan, second stream, join) captured into a CUDA graph on a side stream and replayed on
    new LLRs equals the eager decode of those LLRs bit for bit."""
    H = np.asarray(get_code(code)[0])
    dec = ldpc_amd.get_decoder(H)
    B = 512
    x0 = _llr(H, B, 3.0, seed=11)
    x0[::3, 7] = 0.0
    x1 = _llr(H, B, 2.5, seed=12)
    x1[1::5, 9] = 0.0
    xt = torch.from_numpy(x0).cuda()
    kw = dict(algo="tanh", clamp=20.0, soft="z", want_iters=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):  # warm up: library workspace, auxiliary stream and events exist before capture
            dec.decode(xt, 10, **kw)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = dec.decode(xt, 10, **kw)
    xt.copy_(torch.from_numpy(x1).cuda())
    graph.replay()
    torch.cuda.synchronize()
    ref = dec.decode(torch.from_numpy(x1).cuda(), 10, **kw)
    gen = dec.decode(torch.from_numpy(x1).cuda(), 10, force_generic=True, **kw)
    assert _same(out, ref) and _same(ref, gen)
