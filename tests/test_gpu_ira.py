"""GPU parity of the DVB-S2-structured min-sum kernels (csrc/ira.hip; BASELINE config [4]): bits AND soft z bit
for bit against the C oracle (oracle/ldpc_oracle.c ms_f32, the flooding min-sum the generic kernels also match)
and against the generic CSR kernels on the same batch, at config [4]'s 50 iterations and at the edges: 0 and
1 iterations, exact-zero and negative-zero LLRs (the sign rules of v2c = app - c2v), saturating LLRs, a
batch that is not a multiple of the 8-codeword XCD group, several Infinity-Cache chunk sizes, normalised and
offset min-sum, and the DVB-S2-shaped code with other table addresses.  The reference cannot instantiate a
code of this size (dense E x E masks, masking.py:36-38): parity here is against the oracle."""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import ldpc_amd  # noqa: E402
from ldpc_amd.codes import IRAEncoder, get_code  # noqa: E402


def _llr(code, B, ebn0, seed):
    rng = np.random.default_rng(seed)
    enc = IRAEncoder(code)
    cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
    sigma = np.sqrt(1.0 / (2 * 0.5 * 10 ** (ebn0 / 10)))
    return cw, (-2.0 * ((1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)) / sigma**2).astype(np.float32)


def _decode(dec, x, iters, **kw):
    r = dec.decode(torch.from_numpy(x).cuda(), iters, algo="minsum", soft="z", want_iters=True, **kw)
    torch.cuda.synchronize()
    return r["bits"].cpu().numpy(), r["soft"].cpu().numpy(), r["iters_used"].cpu().numpy()


def _same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.fixture(scope="module")
def dvbs2():
    H, _ = get_code("dvbs2_12")
    return H, ldpc_amd.get_decoder(H)


def test_kernel_path_selection(dvbs2):
    H, dec = dvbs2
    assert dec.kernel_path(dec.params(50, "minsum", 20.0)) == "ira-z360"
    assert dec.kernel_path(dec.params(50, "minsum", 20.0, alpha=0.75, beta=0.5)) == "ira-z360"
    # not (yet) covered by the IRA kernels: the generic CSR kernels take them
    assert dec.kernel_path(dec.params(50, "minsum", 20.0, force_generic=True)) == "generic-csr"
    assert dec.kernel_path(dec.params(50, "minsum", 20.0, early_stop=True)) == "ira-z360"
    assert dec.kernel_path(dec.params(50, "tanh", 20.0)) == "generic-csr"
    wifi = ldpc_amd.get_decoder(get_code("wifi648_12")[0])
    assert wifi.kernel_path(wifi.params(50, "minsum", 20.0)) == "qc-z27"
    peg = ldpc_amd.get_decoder(get_code("peg64_32")[0])
    assert peg.kernel_path(peg.params(5, "minsum", 20.0)) == "generic-csr"


@pytest.mark.parametrize("ebn0", [0.8, 1.2, 1.6])
def test_config4_50it_vs_oracle_bitwise(dvbs2, ebn0):
    """Config [4] itself (50 iterations, clamp 20, plain min-sum) around the waterfall: bits and z bitwise."""
    H, dec = dvbs2
    _, x = _llr(H, 21, ebn0, seed=int(ebn0 * 10))          # 21: not a multiple of the 8-codeword XCD group
    bits, z, used = _decode(dec, x, 50, clamp=20.0)
    ref = oracle.ms_f32(H, x, 50, 20.0)
    assert np.array_equal(bits, ref["bits"])
    assert _same(z, ref["z"])
    assert (used == 50).all()


@pytest.mark.parametrize("alpha,beta,clamp", [(0.75, 0.0, 20.0), (1.0, 0.5, 20.0), (0.8125, 0.25, 6.0)])
def test_normalised_offset_vs_oracle(dvbs2, alpha, beta, clamp):
    H, dec = dvbs2
    _, x = _llr(H, 9, 1.0, seed=3)
    bits, z, _ = _decode(dec, x, 20, clamp=clamp, alpha=alpha, beta=beta)
    ref = oracle.ms_f32(H, x, 20, clamp, alpha, beta)
    assert np.array_equal(bits, ref["bits"]) and _same(z, ref["z"])


@pytest.mark.parametrize("iters", [0, 1, 2, 7])
def test_few_iterations_and_signed_zeros(dvbs2, iters):
    """Exact zeros of both signs and saturating values among the LLRs: the first VN pass must form L + 0
    (a -0 LLR gives +0, as the oracle's app += 0), and v2c = app - c2v keeps the oracle's sign bits."""
    H, dec = dvbs2
    _, x = _llr(H, 10, 1.4, seed=11 + iters)
    rng = np.random.default_rng(iters)
    mask = rng.random(x.shape)
    x[mask < 0.02] = 0.0
    x[(mask >= 0.02) & (mask < 0.04)] = -0.0
    x[(mask >= 0.04) & (mask < 0.045)] = 1e30
    x[(mask >= 0.045) & (mask < 0.05)] = -1e30
    bits, z, _ = _decode(dec, x, iters, clamp=20.0)
    ref = oracle.ms_f32(H, x, iters, 20.0)
    assert np.array_equal(bits, ref["bits"]) and _same(z, ref["z"])


def test_equals_generic_kernels_and_chunking(dvbs2, monkeypatch):
    """The IRA path equals the generic CSR kernels bit for bit on one batch, whatever the Infinity-Cache chunk
    (one pass, 8-codeword chunks with a ragged last chunk, the default)."""
    H, dec = dvbs2
    _, x = _llr(H, 45, 1.3, seed=5)
    gb, gz, _ = _decode(dec, x, 12, clamp=20.0, force_generic=True)
    for budget in ("0", "1", None):
        if budget is None:
            monkeypatch.delenv("LDPC_IRA_BUDGET_MB", raising=False)
        else:
            monkeypatch.setenv("LDPC_IRA_BUDGET_MB", budget)
        bits, z, _ = _decode(dec, x, 12, clamp=20.0)
        assert np.array_equal(bits, gb) and _same(z, gz), budget
    monkeypatch.delenv("LDPC_IRA_BUDGET_MB", raising=False)
    for tpw in ("2", "7", "200"):  # tasks per workgroup: ragged last group, one group per codeword
        monkeypatch.setenv("LDPC_IRA_TPW", tpw)
        bits, z, _ = _decode(dec, x, 12, clamp=20.0)
        assert np.array_equal(bits, gb) and _same(z, gz), tpw
    monkeypatch.delenv("LDPC_IRA_TPW", raising=False)
    for ns in ("1", "2", "3", "4"):  # chunks round-robin over ns streams
        monkeypatch.setenv("LDPC_IRA_STREAMS", ns)
        for budget in ("1", "5", None):
            if budget is None:
                monkeypatch.delenv("LDPC_IRA_BUDGET_MB", raising=False)
            else:
                monkeypatch.setenv("LDPC_IRA_BUDGET_MB", budget)
            bits, z, _ = _decode(dec, x, 12, clamp=20.0)
            assert np.array_equal(bits, gb) and _same(z, gz), (ns, budget)
    monkeypatch.delenv("LDPC_IRA_STREAMS", raising=False)
    monkeypatch.delenv("LDPC_IRA_BUDGET_MB", raising=False)


def test_shaped_code_and_host_pointers():
    """The DVB-S2-shaped code (other table addresses, same degree profile) through host pointers, soft p1."""
    H, _ = get_code("dvbs2s_12")
    dec = ldpc_amd.get_decoder(H)
    assert dec.kernel_path(dec.params(30, "minsum", 20.0)) == "ira-z360"
    _, x = _llr(H, 6, 1.2, seed=9)
    r = dec.decode(x, 30, algo="minsum", clamp=20.0, soft="p1")
    g = dec.decode(x, 30, algo="minsum", clamp=20.0, soft="p1", force_generic=True)
    ref = oracle.ms_f32(H, x, 30, 20.0)
    assert np.array_equal(r["bits"], ref["bits"]) and np.array_equal(r["bits"], g["bits"])
    assert _same(r["soft"], g["soft"])


@pytest.mark.parametrize("ebn0,budget", [(1.0, None), (1.4, "1"), (1.8, None), (2.5, "3")])
def test_early_stop_vs_oracle_bitwise(dvbs2, ebn0, budget, monkeypatch):
    """Early termination (the oracle's ms_f32 early_stop: app_{it+1} tested after each iteration): bits, z and
    iters_used bit for bit against the oracle and the generic kernels, from the waterfall (few converge) to where
    every codeword stops early, over one chunk and over several chunks on two streams."""
    H, dec = dvbs2
    if budget is not None:
        monkeypatch.setenv("LDPC_IRA_BUDGET_MB", budget)
    _, x = _llr(H, 19, ebn0, seed=int(ebn0 * 100))
    bits, z, used = _decode(dec, x, 30, clamp=20.0, early_stop=True)
    ref = oracle.ms_f32(H, x, 30, 20.0, early_stop=True)
    assert np.array_equal(used, ref["iters_used"]), (used, ref["iters_used"])
    assert np.array_equal(bits, ref["bits"]) and _same(z, ref["z"])
    gb, gz, gu = _decode(dec, x, 30, clamp=20.0, early_stop=True, force_generic=True)
    assert np.array_equal(gu, used) and np.array_equal(gb, bits) and _same(gz, z)
    if ebn0 >= 1.8:
        assert (used < 30).all()


def test_host_pointers_with_forked_chunks(dvbs2, monkeypatch):
    """Host pointers (staged through the library's workspace; Decoder.decode and ldpc_amd.decode) with several
    Infinity-Cache chunks on two streams: the forked stream is ordered after the staging copy and joined before
    the copy back."""
    H, dec = dvbs2
    monkeypatch.setenv("LDPC_IRA_BUDGET_MB", "1")           # 8-codeword chunks: 3 chunks over 2 streams
    _, x = _llr(H, 21, 1.3, seed=21)
    r = dec.decode(x, 9, algo="minsum", clamp=20.0, soft="z")
    ref = oracle.ms_f32(H, x, 9, 20.0)
    assert np.array_equal(r["bits"], ref["bits"]) and _same(r["soft"], ref["z"])
    out = ldpc_amd.decode(H, x, 9, algo="minsum", clamp=20.0)
    assert np.array_equal(np.asarray(out), ref["bits"])


def test_one_codeword_and_empty_batch(dvbs2):
    """Batch edges on the IRA path: one codeword (a single XCD group slot, one chunk) bitwise against the oracle
    with and without early stop; an empty batch returns empty outputs without a launch."""
    H, dec = dvbs2
    _, x = _llr(H, 1, 1.6, seed=1)
    for es in (False, True):
        bits, z, used = _decode(dec, x, 12, clamp=20.0, early_stop=es)
        ref = oracle.ms_f32(H, x, 12, 20.0, early_stop=es)
        assert np.array_equal(used, ref["iters_used"]) and np.array_equal(bits, ref["bits"]) and _same(z, ref["z"])
    r = dec.decode(np.zeros((0, H.n), np.float32), 12, algo="minsum", clamp=20.0, soft="z")
    assert r["bits"].shape == (0, H.n) and r["soft"].shape == (0, H.n)


def _shaped_ira(q, G, degs, seed, Z=360):
    """A random IRA code with the DVB-S2 structure: G groups of Z information bits (row degrees `degs`), q rows
    of checks per position; every residue mod q gets the same number of addresses, distinct inside a row."""
    from ldpc_amd.codes import _ira_code
    rng = np.random.default_rng(seed)
    per = sum(degs) // q
    assert per * q == sum(degs)
    left, rows = np.full(q, per), []
    for d in degs:                                        # the d residues with the most addresses left (random ties)
        perm = rng.permutation(q)
        r = perm[np.argsort(-left[perm], kind="stable")[:d]]
        left[r] -= 1
        rows.append(r)
    assert (left == 0).all()
    groups = [r + q * rng.integers(0, Z, size=len(r)) for r in rows]
    k, m = G * Z, q * Z
    return _ira_code(groups, f"ira_q{q}_g{G}", n=k + m, k=k, q=q, Z=Z)


@pytest.mark.parametrize("shape", ["r23_long", "short", "six", "nine"])
def test_other_ira_shapes_vs_oracle(shape):
    """Other IRA shapes through the same kernels: a rate-2/3-shaped normal frame (q = 60, 12 groups of degree 13 —
    the 16-slot variable kernel — and 108 of degree 3; 8 information slots per check), a short one (q = 25, 20
    groups; 4 slots: the 5-slot check kernel), one with 6 slots per check (the 6-slot check kernel) and one with 9
    (the 24-slot check kernel, per-slot branches): bits, z and iteration counts bitwise against the oracle, fixed
    count and early stop."""
    if shape == "r23_long":                                 # _llr's noise is set for rate 1/2: points shifted
        H, pts = _shaped_ira(60, 120, [13] * 12 + [3] * 108, seed=23), ((3.2, False), (4.0, True))
    elif shape == "short":
        H, pts = _shaped_ira(25, 20, [8] * 8 + [3] * 12, seed=7), ((1.0, False), (2.6, True))
    elif shape == "six":
        H, pts = _shaped_ira(20, 20, [8] * 10 + [4] * 10, seed=6), ((1.0, False), (2.6, True))
    else:
        H, pts = _shaped_ira(12, 18, [12] * 6 + [3] * 12, seed=9), ((1.5, False), (3.0, True))
    dec = ldpc_amd.get_decoder(H)
    assert dec.kernel_path(dec.params(20, "minsum", 20.0)) == "ira-z360"
    for ebn0, es in pts:
        _, x = _llr(H, 11, ebn0, seed=31)
        bits, z, used = _decode(dec, x, 20, clamp=20.0, early_stop=es)
        ref = oracle.ms_f32(H, x, 20, 20.0, early_stop=es)
        assert np.array_equal(used, ref["iters_used"]) and np.array_equal(bits, ref["bits"]) and _same(z, ref["z"]), (ebn0, es)


def test_not_ira_when_structure_breaks():
    """A DVB-S2 H with one information edge moved is no longer IRA-structured: the generic kernels take it."""
    H, _ = get_code("dvbs2_12")
    from ldpc_amd.codes import SparseCode
    rp, ci = H.row_ptr.copy(), H.col_idx.copy()
    e = rp[100] + 1                        # an information edge of check 100: move it to a column it lacks
    row = set(ci[rp[100]:rp[101]].tolist())
    new = next(c for c in range(ci[e] + 1, H.k) if c not in row)
    ci[e] = new
    ci[rp[100]:rp[101]].sort()
    broken = SparseCode(H.m, H.n, rp, ci, name="broken")
    dec = ldpc_amd.get_decoder(broken)
    assert dec.kernel_path(dec.params(10, "minsum", 20.0)) == "generic-csr"
