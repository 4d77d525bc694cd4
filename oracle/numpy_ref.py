"""Second, independent restatement of the decoders in numpy (vectorised over codewords, loops over
edges).  TEST INFRASTRUCTURE ONLY: it cross-checks oracle/ldpc_oracle.c on small codes, in particular
for min-sum, which has no reference counterpart to pin it.

tanh-SP follows pytorch/bp/bp.py:43-51, bp_vc.py:16-27, bp_cv.py:22-50; min-sum follows the
specification in oracle/ldpc_oracle.c.
"""
import numpy as np

ZTHR_F32 = np.float32(-1.7881392e-07)


def _graph(H):
    H = np.asarray(H)
    rows, cols = np.nonzero(H)
    m, n = H.shape
    checks = [np.nonzero(rows == c)[0] for c in range(m)]           # check-order edge ids per check
    vars_ = [np.nonzero(cols == v)[0] for v in range(n)]             # ascending check order per var
    return m, n, rows, cols, checks, vars_


def sp(H, llr, iters, clamp, dtype=np.float64):
    m, n, rows, cols, checks, vars_ = _graph(H)
    llr = np.asarray(llr, dtype)
    B, E = llr.shape[0], len(rows)
    x = np.zeros((B, E), dtype)
    pmax = dtype(1 - 1e-7) if dtype == np.float32 else 1 - 1e-7
    half = dtype(0.5)
    for _ in range(iters):
        t = np.empty((B, E), dtype)
        for v in range(n):
            es = vars_[v]
            for k, e in enumerate(es):
                S = np.zeros(B, dtype)
                for u, e2 in enumerate(es):
                    if u != k:
                        S = S + x[:, e2]
                t[:, e] = np.tanh(half * (-llr[:, v] + S))
        for c in range(m):
            es = checks[c]
            for e in es:
                p = np.ones(B, dtype)
                for e2 in es:
                    if e2 != e:
                        p = p * t[:, e2]
                p = np.clip(p, -pmax, pmax)
                y = np.log((dtype(1) + p) / (dtype(1) - p))
                x[:, e] = np.clip(y, -dtype(clamp), dtype(clamp))
    z = np.empty((B, n), dtype)
    for v in range(n):
        S = np.zeros(B, dtype)
        for e in vars_[v]:
            S = S + x[:, e]
        z[:, v] = half * (-llr[:, v] + S)
    return z


def ms(H, llr, iters, clamp, alpha=1.0, beta=0.0):
    """min-sum, float32, exactly the oracle's operation order."""
    m, n, rows, cols, checks, vars_ = _graph(H)
    llr = np.asarray(llr, np.float32)
    B, E = llr.shape[0], len(rows)
    f = np.float32
    c2v = np.zeros((B, E), f)

    def app_of():
        a = -llr.copy()
        for v in range(n):
            for e in vars_[v]:
                a[:, v] = a[:, v] + c2v[:, e]
        return a

    app = app_of()
    for _ in range(iters):
        new = np.empty_like(c2v)
        for c in range(m):
            es = checks[c]
            t = np.stack([app[:, cols[e]] - c2v[:, e] for e in es], axis=1)   # (B, d)
            mag = np.abs(t)
            order = np.argsort(mag, axis=1, kind="stable")
            idx = order[:, 0]
            min1 = np.take_along_axis(mag, order[:, :1], 1)[:, 0]
            min2 = np.take_along_axis(mag, order[:, 1:2], 1)[:, 0] if len(es) > 1 else np.full(B, np.inf, f)
            sgn = (np.signbit(t).sum(axis=1) % 2).astype(bool)
            for k, e in enumerate(es):
                mm = np.where(idx == k, min2, min1).astype(f)
                mm = f(alpha) * mm
                mm = np.maximum(mm - f(beta), f(0))
                mm = np.minimum(mm, f(clamp))
                neg = sgn ^ np.signbit(t[:, k])
                new[:, e] = np.where(neg, -mm, mm)
        c2v = new
        app = app_of()
    return f(0.5) * app
