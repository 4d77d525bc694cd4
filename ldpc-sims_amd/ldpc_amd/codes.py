"""Parity-check matrices, the Tanner-graph layout shared by every decoder, and encoders.

Reference anchors (realjwin/ldpc-sims, read-only at /root/reference):
  * ``pytorch/bp/parity.py:7-47``  — the (64,32) PEG code ``H`` (32x64, 96 edges) and ``G = [I; P]``.
  * ``pytorch/bp/masking.py:84-95`` — edge numbering. ``clookup`` numbers the non-zeros of H row-major
    (the *check-order* edge id, the layout of the reference's ``x`` tensor); ``vlookup`` numbers them
    column-major (*var-order* id, the layout of the VC output).  ``Graph`` keeps exactly that numbering:
    edge id == CSR position, and ``var_edges`` lists, per variable, its check-order edge ids in
    ascending check order (== the var-order id sequence).

The 802.11n tables below are typed in from IEEE 802.11n-2009 Annex R (no network here, nothing in the
reference holds them); ``tests/test_codes.py`` checks their structure (dual-diagonal parity part,
full rank, zero syndrome of encoder output).  Parity for the table contents is therefore *unpinned* by
the reference (SURVEY.md §7 hard part 4).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from functools import lru_cache

import numpy as np

# ---------------------------------------------------------------------------------------------
# (64,32) PEG code of the reference (pytorch/bp/parity.py:7-40): column indices of the 3 ones per
# row.  Data only; tests/test_codes.py compares it against tests/golden/peg64_32.npz, which
# tests/golden/make_golden.py exported from the reference module itself.
_PEG64_ROWS = (
    (0, 16, 32), (0, 17, 33), (1, 16, 34), (1, 18, 35), (2, 17, 36), (2, 19, 37), (3, 18, 38),
    (3, 20, 39), (4, 19, 40), (4, 21, 41), (5, 20, 42), (5, 22, 43), (6, 21, 44), (6, 23, 45),
    (7, 22, 46), (7, 24, 47), (8, 23, 48), (8, 25, 49), (9, 24, 50), (9, 26, 51), (10, 25, 52),
    (10, 27, 53), (11, 26, 54), (11, 28, 55), (12, 27, 56), (12, 29, 57), (13, 28, 58),
    (13, 30, 59), (14, 29, 60), (14, 31, 61), (15, 30, 62), (15, 31, 63),
)


def peg_64_32() -> np.ndarray:
    """The reference's only code: (64,32) PEG, H is 32x64 int (``bp/parity.py:7-40``)."""
    H = np.zeros((32, 64), dtype=np.int64)
    for r, cols in enumerate(_PEG64_ROWS):
        H[r, list(cols)] = 1
    return H


def peg_64_32_generator() -> np.ndarray:
    """``G = [I; P]`` with ``P = H[:, 0:32]`` (``bp/parity.py:42-44``); codeword = G @ info mod 2."""
    H = peg_64_32()
    return np.concatenate([np.eye(32, dtype=np.int64), H[:, 0:32]], axis=0)


# ---------------------------------------------------------------------------------------------
# IEEE 802.11n (HT) LDPC base matrices.  Entry = cyclic right-shift of the ZxZ identity, '-' = null.
_WIFI_TABLES = {
    (648, "1/2"): (27, """
 0  -  -  -  0  0  -  -  0  -  -  0  1  0  -  -  -  -  -  -  -  -  -  -
22  0  -  - 17  -  0  0 12  -  -  -  -  0  0  -  -  -  -  -  -  -  -  -
 6  -  0  - 10  -  -  - 24  -  0  -  -  -  0  0  -  -  -  -  -  -  -  -
 2  -  -  0 20  -  -  - 25  0  -  -  -  -  -  0  0  -  -  -  -  -  -  -
23  -  -  -  3  -  -  -  0  -  9 11  -  -  -  -  0  0  -  -  -  -  -  -
24  - 23  1 17  -  3  - 10  -  -  -  -  -  -  -  -  0  0  -  -  -  -  -
25  -  -  -  8  -  -  -  7 18  -  -  0  -  -  -  -  -  0  0  -  -  -  -
13 24  -  -  0  -  8  -  6  -  -  -  -  -  -  -  -  -  -  0  0  -  -  -
 7 20  - 16 22 10  -  - 23  -  -  -  -  -  -  -  -  -  -  -  0  0  -  -
11  -  -  - 19  -  -  - 13  -  3 17  -  -  -  -  -  -  -  -  -  0  0  -
25  -  8  - 23 18  - 14  9  -  -  -  -  -  -  -  -  -  -  -  -  -  0  0
 3  -  -  - 16  -  -  2 25  5  -  -  1  -  -  -  -  -  -  -  -  -  -  0
"""),
    (1296, "2/3"): (54, """
39 31 22 43  - 40  4  - 11  -  - 50  -  -  -  6  1  0  -  -  -  -  -  -
25 52 41  2  6  - 14  - 34  -  -  - 24  - 37  -  -  0  0  -  -  -  -  -
43 31 29  0 21  - 28  -  -  2  -  -  7  - 17  -  -  -  0  0  -  -  -  -
20 33 48  -  4 13  - 26  -  - 22  -  - 46 42  -  -  -  -  0  0  -  -  -
45  7 18 51 12 25  -  -  - 50  -  -  5  -  -  -  0  -  -  -  0  0  -  -
35 40 32 16  5  -  - 18  -  - 43 51  - 32  -  -  -  -  -  -  -  0  0  -
 9 24 13 22 28  -  - 37  -  - 25  -  - 52  - 13  -  -  -  -  -  -  0  0
32 22  4 21 16  -  -  - 27 28  - 38  -  -  -  8  1  -  -  -  -  -  -  0
"""),
    (1944, "5/6"): (81, """
13 48 80 66  4 74  7 30 76 52 37 60  - 49 73 31 74 73 23  -  1  0  -  -
69 63 74 56 64 77 57 65  6 16 51  - 64  - 68  9 48 62 54 27  -  0  0  -
51 15  0 80 24 25 42 54 44 71 71  9 67 35  - 58  - 29  - 53  0  -  0  0
16 29 36 41 44 56 59 37 50 24  - 65  4 65 52  -  4  - 73 52  1  -  -  0
"""),
}


def _parse_base(text: str) -> np.ndarray:
    rows = [r.split() for r in text.strip().splitlines()]
    return np.array([[-1 if t == "-" else int(t) for t in r] for r in rows], dtype=np.int32)


@dataclass(frozen=True)
class QCCode:
    """A quasi-cyclic code: base matrix of shifts (``-1`` = null block) lifted by ``Z``."""

    base: np.ndarray  # (mb, nb) int32
    Z: int
    name: str = ""

    @property
    def mb(self) -> int:
        return int(self.base.shape[0])

    @property
    def nb(self) -> int:
        return int(self.base.shape[1])

    @property
    def n(self) -> int:
        return self.nb * self.Z

    @property
    def m(self) -> int:
        return self.mb * self.Z

    @property
    def k(self) -> int:
        return self.n - self.m

    def H(self) -> np.ndarray:
        return qc_expand(self.base, self.Z)


def qc_expand(base: np.ndarray, Z: int) -> np.ndarray:
    """Lift a base matrix: block (r, j) with shift s puts a 1 at (r*Z+i, j*Z+(i+s) mod Z)."""
    base = np.asarray(base)
    mb, nb = base.shape
    H = np.zeros((mb * Z, nb * Z), dtype=np.int64)
    i = np.arange(Z)
    for r in range(mb):
        for j in range(nb):
            s = int(base[r, j])
            if s >= 0:
                H[r * Z + i, j * Z + (i + s) % Z] = 1
    return H


def wifi_code(n: int, rate: str) -> QCCode:
    """IEEE 802.11n LDPC code by block length and rate string, e.g. ``wifi_code(648, "1/2")``."""
    try:
        Z, text = _WIFI_TABLES[(int(n), rate)]
    except KeyError:
        raise ValueError(f"802.11n code ({n},{rate}) not embedded; have {sorted(_WIFI_TABLES)}") from None
    return QCCode(_parse_base(text), Z, name=f"wifi{n}_{rate.replace('/', '')}")


def available_codes():
    return ["peg64_32"] + [f"wifi{n}_{r.replace('/', '')}" for (n, r) in sorted(_WIFI_TABLES)] + ["dvbs2_12", "dvbs2s_12"]


def get_code(name: str):
    """Return ``(H, qc)`` for a named code; ``qc`` is the QCCode or ``None``."""
    if name == "peg64_32":
        return peg_64_32(), None
    if name == "dvbs2_12":
        return dvbs2_12(), None
    if name == "dvbs2s_12":
        return dvbs2_shaped(), None
    if name.startswith("wifi"):
        body = name[4:]
        n, r = body.split("_")
        rate = f"{r[0]}/{r[1:]}"
        qc = wifi_code(int(n), rate)
        return qc.H(), qc
    raise ValueError(f"unknown code {name!r}; have {available_codes()}")


# ---------------------------------------------------------------------------------------------
@dataclass
class Graph:
    """CSR (check-major) Tanner graph with the reference's edge numbering.

    ``row_ptr[m+1]``, ``col_idx[E]``: edges of check c are ``row_ptr[c]..row_ptr[c+1]`` with ascending
    variable index (``masking.py:44-47,84-88``).  ``var_ptr[n+1]``, ``var_edges[E]``: the check-order
    edge ids of variable v in ascending check order (``masking.py:52-55,91-95``), so position
    ``var_ptr[v]+t`` is the reference's var-order edge id.
    """

    m: int
    n: int
    row_ptr: np.ndarray
    col_idx: np.ndarray
    var_ptr: np.ndarray
    var_edges: np.ndarray
    edge_check: np.ndarray = field(repr=False, default=None)

    @property
    def E(self) -> int:
        return int(self.col_idx.shape[0])

    @classmethod
    def from_csr(cls, m: int, n: int, row_ptr, col_idx) -> "Graph":
        row_ptr = np.asarray(row_ptr, np.int32)
        col_idx = np.asarray(col_idx, np.int32)
        rows = np.repeat(np.arange(m, dtype=np.int32), np.diff(row_ptr))
        order = np.lexsort((rows, col_idx)).astype(np.int32)   # column-major = ascending check per column
        var_ptr = np.zeros(n + 1, dtype=np.int32)
        np.add.at(var_ptr, col_idx + 1, 1)
        var_ptr = np.cumsum(var_ptr).astype(np.int32)
        return cls(m, n, row_ptr, col_idx, var_ptr, order, rows)

    @classmethod
    def from_H(cls, H) -> "Graph":
        if isinstance(H, SparseCode):
            return cls.from_csr(H.m, H.n, H.row_ptr, H.col_idx)
        H = np.asarray(H)
        if H.ndim != 2:
            raise ValueError("H must be a 2-D 0/1 matrix")
        if not np.isin(H, (0, 1)).all():
            raise ValueError("H must contain only 0/1")
        m, n = H.shape
        rows, cols = np.nonzero(H)  # row-major order == clookup order
        row_ptr = np.zeros(m + 1, dtype=np.int32)
        np.add.at(row_ptr, rows + 1, 1)
        row_ptr = np.cumsum(row_ptr).astype(np.int32)
        col_idx = cols.astype(np.int32)
        # var-order: stable sort of edge ids by column keeps ascending check order within a column
        order = np.argsort(cols, kind="stable").astype(np.int32)
        var_ptr = np.zeros(n + 1, dtype=np.int32)
        np.add.at(var_ptr, cols + 1, 1)
        var_ptr = np.cumsum(var_ptr).astype(np.int32)
        return cls(m, n, row_ptr, col_idx, var_ptr, order, rows.astype(np.int32))

    def check_degrees(self) -> np.ndarray:
        return np.diff(self.row_ptr)

    def var_degrees(self) -> np.ndarray:
        return np.diff(self.var_ptr)

    # ---- weighted BP (bp_vc.py:16-27 with non-unit input_weight / llr_weight) -------------------------
    def weight_offsets(self) -> np.ndarray:
        """wofs[n+1]: start of variable v's d_v x d_v block in one iteration's compact VN weights."""
        d = self.var_degrees().astype(np.int64)
        return np.concatenate([[0], np.cumsum(d * d)])

    def vn_weight_index(self):
        """(target var-order edge, source check-order edge, compact position) of every off-diagonal entry:
        compact[wofs[v] + t*d + u] = input_weight[var_ptr[v]+t][var_edges[var_ptr[v]+u]] (the reference's
        mask_v rows are var-order ids, columns check-order ids, masking.py:101-113)."""
        wofs = self.weight_offsets()
        tgt, src, pos = [], [], []
        for v in range(self.n):
            a, b = int(self.var_ptr[v]), int(self.var_ptr[v + 1])
            d = b - a
            for t in range(d):
                for u in range(d):
                    if u != t:
                        tgt.append(a + t)
                        src.append(int(self.var_edges[a + u]))
                        pos.append(int(wofs[v]) + t * d + u)
        return np.array(tgt, np.int64), np.array(src, np.int64), np.array(pos, np.int64)

    def compact_weights(self, input_weights=None, llr_weights=None, final_input_weight=None,
                        final_llr_weight=None, iters=None):
        """Dense reference weights -> the compact layout the kernels and the oracle read.

        input_weights: per-iteration E x E (the reference's ``layers[i][0].input_weight``, var-order rows,
        check-order columns); llr_weights: per-iteration (1, n); final_input_weight: n x E
        (``final_layer[0].input_weight``); final_llr_weight: (1, n).  Missing = all ones (returned as None).
        """
        out = dict(vn=None, llr=None, fin=None, fin_llr=None)
        if input_weights is not None:
            tgt, src, pos = self.vn_weight_index()
            W = int(self.weight_offsets()[-1])
            vn = np.zeros((len(input_weights), W), np.float64)
            for i, w in enumerate(input_weights):
                vn[i, pos] = np.asarray(w, np.float64)[tgt, src]
            out["vn"] = vn
        if llr_weights is not None:
            out["llr"] = np.stack([np.asarray(w, np.float64).reshape(-1) for w in llr_weights])
        if final_input_weight is not None:
            fw = np.asarray(final_input_weight, np.float64)
            vv = np.repeat(np.arange(self.n), self.var_degrees())
            out["fin"] = fw[vv, self.var_edges]
        if final_llr_weight is not None:
            out["fin_llr"] = np.asarray(final_llr_weight, np.float64).reshape(-1)
        return out


# ---------------------------------------------------------------------------------------------
def _gf2_solve_right(B: np.ndarray, A: np.ndarray) -> np.ndarray:
    """Return X with B @ X = A (mod 2) for square invertible B (uint8 dense, row ops)."""
    m = B.shape[0]
    M = np.concatenate([B, A], axis=1).astype(np.uint8) & 1
    for c in range(m):
        piv = np.nonzero(M[c:, c])[0]
        if piv.size == 0:
            raise np.linalg.LinAlgError("parity part of H is singular over GF(2)")
        p = c + int(piv[0])
        if p != c:
            M[[c, p]] = M[[p, c]]
        hit = np.nonzero(M[:, c])[0]
        hit = hit[hit != c]
        if hit.size:
            M[hit] ^= M[c]
    return M[:, m:]


@lru_cache(maxsize=16)
def _parity_map_cached(key: bytes, shape: tuple) -> np.ndarray:
    H = np.frombuffer(key, dtype=np.uint8).reshape(shape)
    m, n = H.shape
    k = n - m
    return _gf2_solve_right(H[:, k:], H[:, :k])  # (m, k): parity = Pm @ info


def gf2_rank(H) -> int:
    M = (np.asarray(H) & 1).astype(np.uint8).copy()
    r = 0
    rows, cols = M.shape
    for c in range(cols):
        piv = np.nonzero(M[r:, c])[0]
        if piv.size == 0:
            continue
        p = r + int(piv[0])
        if p != r:
            M[[r, p]] = M[[p, r]]
        hit = np.nonzero(M[:, c])[0]
        hit = hit[hit != r]
        if hit.size:
            M[hit] ^= M[r]
        r += 1
        if r == rows:
            break
    return r


class Encoder:
    """Systematic encoder for H = [A | B] with the last m columns invertible (802.11n, PEG).

    codeword = [info ; B^-1 A info] (mod 2), i.e. information bits first — the layout of the
    reference's ``G = [I; P]`` (``bp/parity.py:44``) and of the 802.11n codes.
    """

    def __init__(self, H):
        H = (np.asarray(H) & 1).astype(np.uint8)
        self.m, self.n = H.shape
        self.k = self.n - self.m
        self.P = _parity_map_cached(H.tobytes(), H.shape)  # (m, k) uint8

    def encode(self, info: np.ndarray) -> np.ndarray:
        info = np.asarray(info).astype(np.int64) & 1
        if info.ndim == 1:
            info = info[None, :]
        par = (info @ self.P.T.astype(np.int64)) & 1
        return np.concatenate([info, par], axis=1).astype(np.uint8)

    def generator_parity(self) -> np.ndarray:
        """(k, m) matrix Gp with parity = info @ Gp mod 2 (for device-side encoding)."""
        return self.P.T.copy()


# ---------------------------------------------------------------------------------------------
@dataclass
class SparseCode:
    """A parity-check matrix kept in CSR form only (codes too large for a dense H)."""

    m: int
    n: int
    row_ptr: np.ndarray
    col_idx: np.ndarray
    name: str = ""
    info_groups: np.ndarray = field(default=None, repr=False)   # IRA: [k // 360][deg] check addresses

    @property
    def shape(self):
        return (self.m, self.n)

    @property
    def k(self) -> int:
        return self.n - self.m

    def sum(self) -> int:
        return int(self.col_idx.shape[0])

    def dense(self) -> np.ndarray:
        H = np.zeros((self.m, self.n), np.int64)
        for c in range(self.m):
            H[c, self.col_idx[self.row_ptr[c]:self.row_ptr[c + 1]]] = 1
        return H


def _ira_code(groups, name: str, n: int = 64800, k: int = 32400, q: int = 90, Z: int = 360) -> SparseCode:
    """IRA code of EN 302 307 §5.3.2: information bit i of group g (i = 0..Z-1) is accumulated into parity
    address (x + i*q) mod m for every address x of row g; parity bit c of check c chains with c-1
    (staircase, p_c ^= p_{c-1}).  Returns the check-major CSR with ascending columns."""
    m = n - k
    cols, chks = [], []
    i = np.arange(Z)
    for g, xs in enumerate(groups):
        for x in xs:
            chks.append((int(x) + i * q) % m)
            cols.append(g * Z + i)
    c = np.arange(m)
    chks += [c, c[1:]]
    cols += [k + c, k + c[1:] - 1]
    chks = np.concatenate(chks)
    cols = np.concatenate(cols)
    order = np.lexsort((cols, chks))
    chks, cols = chks[order], cols[order]
    row_ptr = np.zeros(m + 1, np.int64)
    np.add.at(row_ptr, chks + 1, 1)
    row_ptr = np.cumsum(row_ptr).astype(np.int32)
    dmax = max(len(g) for g in groups)
    return SparseCode(m, n, row_ptr, cols.astype(np.int32), name=name,
                      info_groups=np.array([np.pad(np.asarray(g), (0, dmax - len(g)), constant_values=-1)
                                            for g in groups]))


# EN 302 307 (DVB-S2) Annex B, normal frame (n = 64800), rate 1/2: one row of parity-bit accumulator
# addresses per group of 360 information bits; 36 rows of degree 8, then 54 of degree 3.  Typed from the
# standard.  Structural checks (tests/test_codes.py::test_dvbs2_table_structure): every residue mod 90
# appears exactly 5 times (every check: 5 info edges + 2 staircase edges), no repeated edge, girth >= 6
# (no 4-cycle), IRA-encoded codewords have zero syndrome.  The reference cannot instantiate a code this
# size (masking.py:36-38 builds dense E x E masks), so decoding parity on it is UNPINNED against the
# reference; it is pinned against the oracle (bit-exact) like every other code.
_DVBS2_N_12 = """54 9318 14392 27561 26909 10219 2534 8597
55 7263 4635 2530 28130 3033 23830 3651
56 24731 23583 26036 17299 5750 792 9169
57 5811 26154 18653 11551 15447 13685 16264
58 12610 11347 28768 2792 3174 29371 12997
59 16789 16018 21449 6165 21202 15850 3186
60 31016 21449 17618 6213 12166 8334 18212
61 22836 14213 11327 5896 718 11727 9308
62 2091 24941 29966 23634 9013 15587 5444
63 22207 3983 16904 28534 21415 27524 25912
64 25687 4501 22193 14665 14798 16158 5491
65 4520 17094 23397 4264 22370 16941 21526
66 10490 6182 32370 9597 30841 25954 2762
67 22120 22865 29870 15147 13668 14955 19235
68 6689 18408 18346 9918 25746 5443 20645
69 29982 12529 13858 4746 30370 10023 24828
70 1262 28032 29888 13063 24033 21951 7863
71 6594 29642 31451 14831 9509 9335 31552
72 1358 6454 16633 20354 24598 624 5265
73 19529 295 18011 3080 13364 8032 15323
74 11981 1510 7960 21462 9129 11370 25741
75 9276 29656 4543 30699 20646 21921 28050
76 15975 25634 5520 31119 13715 21949 19605
77 18688 4608 31755 30165 13103 10706 29224
78 21514 23117 12245 26035 31656 25631 30699
79 9674 24966 31285 29908 17042 24588 31857
80 21856 27777 29919 27000 14897 11409 7122
81 29773 23310 263 4877 28622 20545 22092
82 15605 5651 21864 3967 14419 22757 15896
83 30145 1759 10139 29223 26086 10556 5098
84 18815 16575 2936 24457 26738 6030 505
85 30326 22298 27562 20131 26390 6247 24791
86 928 29246 21246 12400 15311 32309 18608
87 20314 6025 26689 16302 2296 3244 19613
88 6237 11943 22851 15642 23857 15112 20947
89 26403 25168 19038 18384 8882 12719 7093
0 14567 24965
1 3908 100
2 10279 240
3 24102 764
4 12383 4173
5 13861 15918
6 21327 1046
7 5288 14579
8 28158 8069
9 16583 11098
10 16681 28363
11 13980 24725
12 32169 17989
13 10907 2767
14 21557 3818
15 26676 12422
16 7676 8754
17 14905 20232
18 15719 24646
19 31942 8589
20 19978 27197
21 27060 15071
22 6071 26649
23 10393 11176
24 9597 13370
25 7081 17677
26 1433 19513
27 26925 9014
28 19202 8900
29 18152 30647
30 20803 1737
31 11804 25221
32 31683 17783
33 29694 9345
34 12280 26611
35 6526 26122
36 26165 11241
37 7666 26962
38 16290 8480
39 11774 10120
40 30051 30426
41 1335 15424
42 6865 17742
43 31779 12489
44 32120 21001
45 14508 6996
46 979 25024
47 4554 21896
48 7989 21777
49 4972 20661
50 6612 2730
51 12742 4418
52 29194 595
53 19267 20113"""


@lru_cache(maxsize=1)
def dvbs2_12() -> SparseCode:
    """DVB-S2 normal-frame rate-1/2 LDPC code (n = 64800, k = 32400, E = 226,799): BASELINE config [4]."""
    groups = [np.array(list(map(int, line.split())), np.int64) for line in _DVBS2_N_12.splitlines()]
    return _ira_code(groups, "dvbs2_12")


def dvbs2_shaped(seed: int = 2019) -> SparseCode:
    """A DVB-S2-SHAPED normal-frame rate-1/2 IRA code: the structure, degree profile and edge count
    (E = 226,799) of :func:`dvbs2_12` (n = 64800, k = 32400, q = 90, 36 rows of degree 8, 54 of degree 3)
    with seeded pseudo-random addresses.  Kept as a second large test code (no 802.11n-like regularity).

    Each residue class mod q receives exactly 5 addresses, distinct inside a row, as in the standard."""
    q, Z = 90, 360
    rng = np.random.default_rng(seed)
    degs = [8] * 36 + [3] * 54
    while True:
        pool = np.repeat(np.arange(q), 5)
        rng.shuffle(pool)
        rows, pos, ok = [], 0, True
        for d in degs:
            r = pool[pos:pos + d]
            pos += d
            if len(set(r.tolist())) != d:
                ok = False
                break
            rows.append(r)
        if ok:
            break
    groups = [r + q * rng.integers(0, Z, size=len(r)) for r in rows]
    return _ira_code(groups, "dvbs2s_12")


class IRAEncoder:
    """Systematic encoder for a SparseCode with staircase parity (info first, then p_0..p_{m-1}):
    p_c = p_{c-1} xor (sum of the info bits of check c)."""

    def __init__(self, code: SparseCode):
        self.code = code
        self.m, self.n, self.k = code.m, code.n, code.k
        rp, ci = code.row_ptr, code.col_idx
        chk = np.repeat(np.arange(self.m), np.diff(rp))
        info = ci < self.k
        self._chk, self._col = chk[info], ci[info]

    def encode(self, info_bits: np.ndarray) -> np.ndarray:
        info_bits = np.atleast_2d(np.asarray(info_bits)).astype(np.uint8) & 1
        B = info_bits.shape[0]
        s = np.zeros((B, self.m), np.int64)
        np.add.at(s.T, self._chk, info_bits[:, self._col].T)
        par = np.cumsum(s, axis=1) & 1
        return np.concatenate([info_bits, par.astype(np.uint8)], axis=1)
