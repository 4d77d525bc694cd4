"""BASELINE config [1] exactly as bench.py decodes it: (648,1/2), min-sum, 50 iterations, clamp 20, B = 65,536
codewords generated on device (ldpc_random_bits -> DeviceEncoder -> ldpc_awgn_llr, bench.py:96-117) at
Eb/N0 points of the bench sweep, one launch through ldpc_decode_ex with a caller workspace on the current
stream.  Checked against the oracle (oracle/ldpc_oracle.c ms_f32) bit for bit — hard bits and soft z — on
1,024 rows spread over the batch, and the on-device error counters (ldpc_count_errors, the bench's BER/BLER
numerators) against counts recomputed on the host from the full decoded batch."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd import _abi  # noqa: E402
from ldpc_amd.synth import DeviceEncoder  # noqa: E402


@pytest.mark.parametrize("ebn0", [1.5, 2.5, 4.0])
def test_bench_config1_decode_and_counts(ebn0):
    H, _ = ldpc_amd.get_code("wifi648_12")
    m, n = H.shape
    k, B, iters, clamp, seed = n - m, 65536, 50, 20.0, 2024
    dec = ldpc_amd.get_decoder(H, 0)
    lib = _abi.load()
    st = torch.cuda.current_stream().cuda_stream
    info = torch.empty((B, k), dtype=torch.uint8, device="cuda")
    _abi.check(lib.ldpc_random_bits(info.data_ptr(), B, k, seed, 0, st))
    cw = DeviceEncoder(H, torch.device("cuda", 0)).encode(info)
    x = torch.empty((B, n), dtype=torch.float32, device="cuda")
    sigma = float(np.sqrt(1.0 / (2.0 * 0.5 * 10.0 ** (ebn0 / 10.0))))
    _abi.check(lib.ldpc_awgn_llr(cw.data_ptr(), x.data_ptr(), B, n, sigma, seed * 1000 + 3, 0, st))
    p = dec.params(iters, "minsum", clamp, 1.0, 0.0, False, "f32", "z", device_ptrs=True)
    wsb = dec.workspace_bytes(B, p)
    ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device="cuda")
    bits = torch.empty((B, n), dtype=torch.uint8, device="cuda")
    z = torch.empty((B, n), dtype=torch.float32, device="cuda")
    _abi.check(lib.ldpc_decode_ex(dec._h, x.data_ptr(), B, p, bits.data_ptr(), z.data_ptr(), None, ws.data_ptr(), wsb, st))
    counts = torch.zeros(3, dtype=torch.int64, device="cuda")
    _abi.check(lib.ldpc_count_errors(bits.data_ptr(), cw.data_ptr(), B, n, k, counts.data_ptr(), st))
    torch.cuda.synchronize()
    assert dec.qc_z == 27   # the register-resident QC kernel, as in the bench line

    rows = np.unique(np.r_[0:256, np.linspace(256, B - 257, 512).astype(np.int64), B - 256:B])
    llr = x[torch.from_numpy(rows).cuda()].cpu().numpy()
    ref = oracle.ms_f32(H, llr, iters, clamp, 1.0, 0.0)
    assert np.array_equal(bits.cpu().numpy()[rows], ref["bits"])
    assert np.array_equal(z.cpu().numpy()[rows].view(np.uint32), ref["z"].view(np.uint32))

    b, c = bits.cpu().numpy(), cw.cpu().numpy()
    err = b != c
    assert counts.cpu().tolist() == [int(err[:, :k].sum()), int(err.any(1).sum()), B]
    if ebn0 <= 1.5:
        assert counts[1].item() > 0   # the counters see errors at the low end of the sweep
