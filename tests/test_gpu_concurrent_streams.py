"""Decodes issued on several streams at once, no synchronisation between them: every result equals the same
decode run alone.  Covers the paths that fork work onto the library's own streams — the tanh-SP zero pass (the
a == 1 rule's kernel on an auxiliary stream, joined back by event) and the IRA path's Infinity-Cache chunks
(round-robin over its stream pool) — interleaved with each other and with the register min-sum and packed
5-bit kernels, so a missing fork or join, or a workspace shared across calls, shows up as a difference."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd.codes import Encoder, IRAEncoder, get_code  # noqa: E402


def _llr(H, enc, B, ebn0, seed, erase=0.0):
    rng = np.random.default_rng(seed)
    cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
    sigma = np.sqrt(1.0 / (10 ** (ebn0 / 10)))
    x = (-2.0 * ((1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)) / sigma**2).astype(np.float32)
    if erase:
        x[rng.random(x.shape) < erase] = 0.0
    return torch.from_numpy(x).cuda()


def test_interleaved_streams_equal_serial(monkeypatch):
    monkeypatch.setenv("LDPC_IRA_BUDGET_MB", "2")       # several IRA chunks per decode
    jobs = []
    for name, algo, kw, B, erase in [
        ("wifi648_12", "tanh", dict(clamp=10.0), 300, 0.02),
        ("wifi1944_56", "tanh", dict(clamp=20.0), 200, 0.01),
        ("wifi1296_23", "qminsum", dict(qstep=1.0, early_stop=True), 500, 0.0),
        ("wifi648_12", "minsum", dict(clamp=20.0), 700, 0.05),
        ("dvbs2_12", "minsum", dict(clamp=20.0), 9, 0.0),
        ("dvbs2_12", "minsum", dict(clamp=20.0, early_stop=True), 7, 0.0),
    ]:
        H, _ = get_code(name)
        enc = IRAEncoder(H) if name.startswith("dvbs2") else Encoder(H)
        dec = ldpc_amd.get_decoder(H)
        for rep in range(2):
            jobs.append((dec, _llr(H, enc, B, 1.5 + rep, seed=len(jobs), erase=erase), algo, kw))
    iters = 12
    serial = []
    for dec, x, algo, kw in jobs:
        r = dec.decode(x, iters, algo=algo, soft="z", want_iters=True, **kw)
        torch.cuda.synchronize()
        serial.append({k: v.clone() for k, v in r.items() if v is not None})
    streams = [torch.cuda.Stream() for _ in range(3)]
    for rnd in range(2):
        order = np.random.default_rng(rnd).permutation(len(jobs))
        outs = [None] * len(jobs)
        for i, j in enumerate(order):
            dec, x, algo, kw = jobs[j]
            outs[j] = dec.decode(x, iters, algo=algo, soft="z", want_iters=True, stream=streams[i % 3], **kw)
        torch.cuda.synchronize()
        for j, (r, s) in enumerate(zip(outs, serial)):
            assert torch.equal(r["bits"], s["bits"]), (rnd, j)
            assert torch.equal(r["soft"].view(torch.int32), s["soft"].view(torch.int32)), (rnd, j)
            assert torch.equal(r["iters_used"], s["iters_used"]), (rnd, j)


def test_more_caller_streams_than_auxiliary_sets(monkeypatch):
    """The library keeps at most 16 auxiliary-stream sets per host thread, one per caller stream (csrc/qc.hip
    aux_get); a 17th caller stream evicts the least recently used set while earlier decodes may still run on it.
    Decodes forked from 20 caller streams, twice round, still equal the serial decodes."""
    monkeypatch.setenv("LDPC_IRA_BUDGET_MB", "2")
    jobs = []
    for name, B in (("wifi648_12", 200), ("dvbs2_12", 5)):
        H, _ = get_code(name)
        enc = IRAEncoder(H) if name.startswith("dvbs2") else Encoder(H)
        dec = ldpc_amd.get_decoder(H)
        algo, kw = ("tanh", dict(clamp=10.0)) if name == "wifi648_12" else ("minsum", dict(clamp=20.0))
        for rep in range(3):
            jobs.append((dec, _llr(H, enc, B, 1.0 + rep, seed=100 + len(jobs), erase=0.02), algo, kw))
    iters = 8
    serial = []
    for dec, x, algo, kw in jobs:
        serial.append(dec.decode(x, iters, algo=algo, soft="z", **kw)["soft"].clone())
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(20)]
    outs = []
    for rnd in range(2):
        for i, s in enumerate(streams):
            j = (i + rnd) % len(jobs)
            dec, x, algo, kw = jobs[j]
            outs.append((j, dec.decode(x, iters, algo=algo, soft="z", stream=s, **kw)["soft"]))
    torch.cuda.synchronize()
    for k, (j, z) in enumerate(outs):
        assert torch.equal(z.view(torch.int32), serial[j].view(torch.int32)), (k, j)
