import os

import numpy as np
import pytest

from conftest import GOLDEN
from ldpc_amd.codes import Encoder, Graph, gf2_rank, peg_64_32, peg_64_32_generator, qc_expand, wifi_code


def test_peg_matches_reference_fixture():
    d = np.load(os.path.join(GOLDEN, "peg64_32.npz"))
    assert np.array_equal(peg_64_32(), d["H"])
    assert np.array_equal(peg_64_32_generator(), d["G"])


def test_graph_numbering_is_reference_clookup_vlookup():
    """masking.py:84-95: check-order ids = row-major nonzeros; var-order = column-major."""
    H = peg_64_32()
    g = Graph.from_H(H)
    rows, cols = np.nonzero(H)
    assert np.array_equal(g.col_idx, cols)
    # var-order sequence of check-order ids == column-major enumeration of the nonzeros
    rc = [(r, c) for r, c in zip(rows, cols)]
    colmajor = sorted(range(len(rc)), key=lambda e: (rc[e][1], rc[e][0]))
    assert np.array_equal(g.var_edges, colmajor)
    assert g.E == 96 and g.m == 32 and g.n == 64


@pytest.mark.parametrize("n,rate,Z,E,k", [(648, "1/2", 27, 2376, 324), (1296, "2/3", 54, 4752, 864),
                                          (1944, "5/6", 81, 6399, 1620)])
def test_wifi_tables_structure(n, rate, Z, E, k):
    q = wifi_code(n, rate)
    H = q.H()
    assert q.Z == Z and q.n == n and q.k == k and int(H.sum()) == E
    mb, nb = q.base.shape
    kb = nb - mb
    # dual-diagonal parity part: h_b column (x, ..., 0, ..., x) and identity staircase
    hb = q.base[:, kb]
    nz = np.nonzero(hb >= 0)[0]
    assert len(nz) == 3 and nz[0] == 0 and nz[-1] == mb - 1 and hb[0] == hb[-1] and hb[nz[1]] == 0
    for r in range(mb):
        for j in range(kb + 1, nb):
            c = j - kb - 1
            assert (q.base[r, j] == 0) == (r in (c, c + 1)) and (q.base[r, j] in (-1, 0))
    assert gf2_rank(H) == mb * Z
    enc = Encoder(H)
    info = np.random.default_rng(1).integers(0, 2, size=(8, enc.k))
    cw = enc.encode(info)
    assert np.array_equal(cw[:, :enc.k], info)
    assert not ((H @ cw.T.astype(np.int64)) % 2).any()


def test_qc_expand_shift_convention():
    H = qc_expand(np.array([[1]]), 4)
    assert H[0, 1] == 1 and H[3, 0] == 1 and H.sum() == 4


def test_graph_rejects_non_binary():
    with pytest.raises(ValueError):
        Graph.from_H(np.array([[0, 2]]))


def test_dvbs2_shaped_structure_and_encoder():
    from ldpc_amd.codes import IRAEncoder, dvbs2_shaped
    c = dvbs2_shaped()
    g = Graph.from_H(c)
    assert (c.m, c.n, g.E) == (32400, 64800, 226799)            # EN 302 307 normal frame, rate 1/2
    dc = np.bincount(g.check_degrees())
    assert dc[7] == 32399 and dc[6] == 1
    dv = np.bincount(g.var_degrees())
    assert dv[8] == 12960 and dv[3] == 19440 and dv[2] == 32399 and dv[1] == 1
    cw = IRAEncoder(c).encode(np.random.default_rng(0).integers(0, 2, size=(2, c.k)))
    for row in cw:
        assert not (np.add.reduceat(row[c.col_idx].astype(np.int64), c.row_ptr[:-1]) % 2).any()


def test_dvbs2_table_structure():
    """EN 302 307 rate-1/2 table (codes._DVBS2_N_12): structural checks that catch a mistyped address.
    The reference cannot build a code this size (masking.py:36-38), so its contents are unpinned."""
    from collections import Counter
    from ldpc_amd.codes import IRAEncoder, _DVBS2_N_12, dvbs2_12
    rows = [list(map(int, ln.split())) for ln in _DVBS2_N_12.splitlines()]
    assert [len(r) for r in rows] == [8] * 36 + [3] * 54
    assert all(0 <= x < 32400 for r in rows for x in r)
    # the first address of each row is its own residue class (54..89, then 0..53)
    assert [r[0] for r in rows] == list(range(54, 90)) + list(range(54))
    # every residue class mod q = 90 receives exactly 5 addresses -> every check has 5 info edges
    assert set(Counter(x % 90 for r in rows for x in r).values()) == {5}
    c = dvbs2_12()
    g = Graph.from_H(c)
    assert (c.m, c.n, g.E) == (32400, 64800, 226799)
    dc = np.bincount(g.check_degrees())
    assert dc[7] == 32399 and dc[6] == 1
    dv = np.bincount(g.var_degrees())
    assert dv[8] == 12960 and dv[3] == 19440 and dv[2] == 32399 and dv[1] == 1
    # no repeated edge, no 4-cycle (two columns sharing two checks): girth >= 6
    key = g.edge_check.astype(np.int64) * c.n + g.col_idx
    assert len(np.unique(key)) == g.E
    pairs = []
    for cc in range(c.m):
        v = g.col_idx[g.row_ptr[cc]:g.row_ptr[cc + 1]].astype(np.int64)
        a, b = np.triu_indices(len(v), 1)
        pairs.append(v[a] * c.n + v[b])
    p = np.concatenate(pairs)
    assert len(np.unique(p)) == len(p)
    cw = IRAEncoder(c).encode(np.random.default_rng(1).integers(0, 2, size=(2, c.k)))
    for row in cw:
        assert not (np.add.reduceat(row[c.col_idx].astype(np.int64), c.row_ptr[:-1]) % 2).any()
