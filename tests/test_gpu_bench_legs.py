"""BASELINE configs [2], [3] and [4] exactly as bench.py's side legs decode them (bench.LEGS / bench.Workload: the
data generated on device at the leg's full batch, one launch per point through ldpc_decode_ex with the leg's
parameters), checked at full size:

* config [2] (1944,5/6) tanh-SP 50 it on 16-QAM OFDM LLRs, B = 32,768: the bench launch's bits equal the register
  kernel's and the generic CSR kernels' over the WHOLE batch, soft z bitwise between the two kernel families
  (the (D, S) arithmetic is specified operation for operation; the oracle comparison is test_gpu_config2.py);
* config [3] (1296,2/3) 5-bit min-sum <= 20 it early stop, B = 65,536: bits, z (= APP / 2) and iteration counts
  bitwise vs the oracle's integer restatement (oracle.qms) on 1,024 rows spread over the batch;
* config [4] DVB-S2 (EN 302 307) 64800 rate 1/2 min-sum 50 it, B = 4,096: bits and z bitwise vs the oracle on 16
  rows spread over the batch;
and for every leg the on-device error counters (the legs' BER/BLER numerators) equal host recounts of the full
decoded batch."""
import argparse
import os
import sys

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ldpc_amd import _abi  # noqa: E402


def _workload(name):
    la = bench.leg_args(name, argparse.Namespace(seed=2024, leg_batch_scale=1.0))
    return la, bench.Workload(la, 0, 0)


def _counts_match(wl, point):
    lib = _abi.load()
    wl.step(wl.llrs[point])
    counts = torch.zeros(3, dtype=torch.int64, device="cuda")
    _abi.check(lib.ldpc_count_errors(wl.bits.data_ptr(), wl.cw.data_ptr(), wl.B, wl.n, wl.k, counts.data_ptr(),
                                     wl.stream.cuda_stream))
    torch.cuda.synchronize()
    err = wl.bits.cpu().numpy() != wl.cw.cpu().numpy()
    assert counts.cpu().tolist() == [int(err[:, :wl.k].sum()), int(err.any(1).sum()), wl.B]
    return wl.bits.clone()


def _rows(B, k):
    return np.unique(np.linspace(0, B - 1, k).astype(np.int64))


def test_config2_leg_full_batch_kernels_agree():
    la, wl = _workload("config2")
    assert wl.B == 32768 and la.iters == 50 and la.mod == "16qam-ofdm" and wl.kpath == "qc-z81"
    i = 5                                                    # Eb/N0 6.5 dB: the waterfall (BLER ~0.1)
    bench_bits = _counts_match(wl, i)
    x = wl.llrs[i]
    a = wl.dec.decode(x, la.iters, algo="tanh", clamp=la.clamp, soft="z")
    g = wl.dec.decode(x, la.iters, algo="tanh", clamp=la.clamp, soft="z", force_generic=True)
    assert torch.equal(bench_bits, a["bits"]) and torch.equal(a["bits"], g["bits"])
    assert torch.equal(a["soft"].view(torch.int32), g["soft"].view(torch.int32))
    bler = float((a["bits"] != wl.cw).any(1).float().mean())
    assert 0.0 < bler < 1.0                                  # a point with both decoded and failing codewords
    wl.free()


def test_config3_leg_full_batch_vs_oracle():
    la, wl = _workload("config3")
    assert wl.B == 65536 and la.iters == 20 and la.early_stop and wl.kpath == "qc-z54"
    for i in (3, 5, 8):                                      # Eb/N0 1.5 / 2.5 / 4 dB: failing, waterfall, converging
        bench_bits = _counts_match(wl, i)
        x = wl.llrs[i]
        r = wl.dec.decode(x, la.iters, algo="qminsum", qstep=la.qstep, early_stop=True, soft="z", want_iters=True)
        assert torch.equal(bench_bits, r["bits"])
        rows = _rows(wl.B, 1024)
        llr = x[torch.from_numpy(rows).cuda()].cpu().numpy()
        q = np.clip(np.rint(llr * (np.float32(1.0) / np.float32(la.qstep))), -15, 15).astype(np.int8)
        ref = oracle.qms(wl.H, q, la.iters, 15, 127, 0, early_stop=True)
        assert np.array_equal(r["bits"].cpu().numpy()[rows], ref["bits"])
        assert np.array_equal(r["iters_used"].cpu().numpy()[rows], ref["iters_used"])
        assert np.array_equal(r["soft"].cpu().numpy()[rows], (0.5 * ref["app"]).astype(np.float32))
    wl.free()


def test_config4_leg_full_batch_vs_oracle():
    la, wl = _workload("config4")
    assert wl.B == 4096 and la.iters == 50 and wl.kpath == "ira-z360"
    i = 3                                                    # Eb/N0 1.5 dB: the waterfall
    bench_bits = _counts_match(wl, i)
    x = wl.llrs[i]
    r = wl.dec.decode(x, la.iters, algo="minsum", clamp=la.clamp, soft="z")
    assert torch.equal(bench_bits, r["bits"])
    rows = _rows(wl.B, 16)
    llr = x[torch.from_numpy(rows).cuda()].cpu().numpy()
    ref = oracle.ms_f32(wl.H, llr, la.iters, la.clamp, 1.0, 0.0)
    assert np.array_equal(r["bits"].cpu().numpy()[rows], ref["bits"])
    assert np.array_equal(r["soft"].cpu().numpy()[rows].view(np.uint32), ref["z"].view(np.uint32))
    wl.free()
