"""cn_ds_row (csrc/common.h) at block sizes on the shared-T boundary ((d - 1) % BLOCK == 0), off it and as one
block, with and without the a == 1 rule: every blocked form equals the one-block form bit for bit (ADVICE r4:
the boundary case read an unset T before the fix; shipped settings — d = 20 in blocks of 7 or one block — never
reach it).  Test-only kernels: tests/kern/cn_rows.hip, built by build.py build_test_kernels."""
import ctypes
import os

import numpy as np
import pytest

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kern", "libcnrows.so")
CMAX2 = np.float32(min(np.float32(20.0) * np.float32(1.4426950408889634), 24.0))  # sp_cmax2(20)
CASES = [(14, 13), (15, 7), (15, 5), (20, 19), (20, 7), (20, 10)]  # (d, BLOCK); boundary: 14/13, 15/7, 20/19


def _lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run python ldpc-sims_amd/build.py (build_test_kernels)")
    L = ctypes.CDLL(LIB)
    L.cnrows_supported.argtypes = [ctypes.c_int, ctypes.c_int]
    L.cnrows_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, ctypes.c_float]
    return L


def _rows(d, n, seed):
    """signed a-values: a = exp(-|s|) for |s| spread over [0, 30] (incl. a == 1, s = +-0) and random signs"""
    rng = np.random.default_rng(seed)
    s = rng.exponential(3.0, size=(n, d)).astype(np.float32)
    s[rng.random((n, d)) < 0.03] = 0.0              # a == 1 edges (several per row in some rows)
    s[rng.random((n, d)) < 0.02] = 30.0             # tiny a
    a = np.exp(-s.astype(np.float64)).astype(np.float32)
    sign = np.where(rng.random((n, d)) < 0.5, -1.0, 1.0).astype(np.float32)
    return np.ascontiguousarray(a * sign)


def _run(L, g, d, block, fix):
    out = np.empty_like(g)
    rc = L.cnrows_run(g.ctypes.data, out.ctypes.data, g.shape[0], d, block, int(fix), CMAX2)
    assert rc == 0, f"cnrows_run({d}, {block}, fix={fix}) = {rc}"
    return out


def test_test_kernel_library_exports():
    """(CPU) the test kernel library loads and instantiates every case plus the one-block forms"""
    L = _lib()
    for d, b in CASES:
        assert L.cnrows_supported(d, b) and L.cnrows_supported(d, d)
    assert not L.cnrows_supported(20, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("fix", [False, True])
@pytest.mark.parametrize("d,block", CASES)
def test_blocked_rows_equal_one_block(d, block, fix):
    L = _lib()
    g = _rows(d, 4096, seed=d * 100 + block)
    ref = _run(L, g, d, d, fix)
    got = _run(L, g, d, block, fix)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
        f"d={d} BLOCK={block} fix={fix}: {(got.view(np.uint32) != ref.view(np.uint32)).sum()} outputs differ"
    assert np.isfinite(ref).all()
    if fix:  # a row with two or more a == 1 edges: every output is +-0
        two = (np.abs(g) == 1.0).sum(axis=1) >= 2
        assert two.any() and (ref[two] == 0.0).all()
