/*
 * ldpc_oracle.c — CPU ORACLE for the LDPC belief-propagation hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only
 * as the checker / CPU comparator.  The product path (ldpc-sims_amd/, libldpc_hip.so) never calls it.
 *
 * It restates, edge by edge, what the reference's dense-mask network computes
 * (realjwin/ldpc-sims @ /root/reference/pytorch):
 *
 *   bp/bp.py:43-51   forward: for it in iters: x = CV(tanh(VC([x, -llr]))).clamp(+-clamp)
 *                    then p1 = 1 - sigmoid(VC_final([x, -llr]))
 *   bp/bp_vc.py:16-27 VC: v2c[e=(c,v)] = 0.5 * (L_v + sum_{c' != c} x[(c',v)])   (L = -llr)
 *                    computed there as a masked mm; every mask weight is exactly 1, so the value is the
 *                    plain sum, accumulated here in ascending check order (the mm's k order).
 *   bp/bp_cv.py:22-50 CV: p = prod_{v' != v} tanh(v2c[(c,v')]); p = clamp(p, +-(1-1e-7));
 *                    x = log((1+p)/(1-p))
 *   ofdm/ofdm_functions.py:161  bits = np.round(p1): bit 1 iff p1 > 0.5 (ties -> 0).  In fp32 that is
 *                    exactly z <= -1.7881392e-07 (0xb43fffff) for torch 2.10's CPU sigmoid; measured
 *                    bit-pattern by bit-pattern in this container (see DESIGN.md "hard decision").
 *
 * Edge numbering is the reference's check-order id (bp/masking.py:84-88): CSR position.
 *
 * Min-sum (ldpc_ms_*) is NOT in the reference: its specification lives here and in
 * DESIGN.md, and the GPU kernels must match it bit for bit.  Parity of min-sum against the reference is
 * unpinned by construction.
 *
 *   APP_v = L_v + sum_{e in v, ascending check} c2v[e]           (c2v = 0 before iteration 0)
 *   v2c_e = APP_v - c2v[e]
 *   check c: min1 <= min2 the two smallest |v2c| (idx = first edge attaining min1), sgn = xor of sign bits
 *   c2v[e] = (sgn ^ signbit(v2c_e)) ? -mag : mag,  mag = min(clamp, max(alpha*m - beta, 0)),
 *            m = (e == idx) ? min2 : min1
 *   after the last iteration: z_v = 0.5 * APP_v, bit = z_v <= ZTHR (same rule as tanh-SP).
 *   early stop (flag): after each iteration's APP, stop the codeword when H*bits = 0.
 *
 * Quantized min-sum (ldpc_qms_*): integer LLRs in [-qmax, qmax] (the caller quantizes), integer messages
 * saturated to +-qmax, APP saturated to +-app_max, offset beta (integer), no alpha; bit = APP < 0.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ZTHR_F32 (-1.7881392e-07f)                    /* 0xb43fffff */
#define ZTHR_F64 (-3.3306690738754696e-16)            /* -1.5 * 2^-52 */
#define PMAX_F32 ((float)(1.0 - 1e-7))                /* torch casts the python bound to fp32 */
#define PMAX_F64 (1.0 - 1e-7)

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

typedef struct {
    int m, n, E;
    const int32_t *row_ptr, *col_idx, *var_ptr, *var_edges;
} graph_t;

/* Weighted BP (bp_vc.py:16-27 with non-unit input_weight / llr_weight): compact layout, per iteration
 *   vn[it*W + wofs[v] + t*d_v + u]  weight of var-slot u's c2v into var-slot t's v2c (u != t; slot = position in
 *                                   var_edges, ascending check), W = sum_v d_v^2, wofs[v] = sum_{v'<v} d_v'^2
 *   lw[it*n + v]                    llr_weight of variable v
 *   fin[var_ptr[v] + u], flw[v]     the final layer's weights
 * v2c = 0.5 * (lw*L + sum_{u != t, ascending} w_tu * x_u) — the masked mm of bp_vc.py:19 and :24,27. */
typedef struct {
    const void *vn, *lw, *fin, *flw;
    const int64_t* wofs;
    int64_t W;
} wts_t;

/* ------------------------------------------------------------------------------------------ */
/* tanh sum-product, fp32 (bp/bp.py:43-51, bp_vc.py:16-27, bp_cv.py:22-50)                      */
static int syndrome_ok(const graph_t* g, const uint8_t* bits);

/* The check-node rule evaluated in the (D, S) form ("stable" mode: what the GPU kernels compute).
 *
 * Mathematically the same function as bp_cv.py:38-50: with s the full-LLR v2c argument (v2c = tanh(s/2),
 * bp_vc.py:27 + bp.py:29) write a = exp(-|s|), so |tanh(s/2)| = (1-a)/(1+a).  For a set of edges let
 * P+ = prod(1+a), P- = prod(1-a); D = P+ - P-, S = P+ + P- (up to a common positive factor).  Then
 * |p| = |prod tanh| = (S-D)/(S+D) and log((1+|p|)/(1-|p|)) = log(S/D).  Adding one edge (a, 1):
 * D' = D + a*S, S' = S + a*D; joining two sets: D = Dp*Sq + Sp*Dq, S = Sp*Sq + Dp*Dq (each one product and one
 * fma: D = fma(Dp, Sq, Sp*Dq), S = fma(Dp, Dq, Sp*Sq), as the kernels' ds_join_out) — sums of positive
 * terms only, so every step is accurate to an ulp, where the reference's fp32 form loses digits near |p| -> 1
 * (1-p cancels; one ulp of tanh near 1 is a 1e-4..1e-3 error in log).  Exclusive (D, S) per edge from prefix
 * and suffix sets, O(d) per check.  The clamp |p| <= 1-1e-7 is S/D <= RMAX = (1+pmax)/(1-pmax) (fp32:
 * 16777215 = the reference's fp32 bound exactly), then the caller's clamp; sign = xor of the others' signs.
 * An s of +-0 gives a = 1 — the reference's tanh(0) = 0 makes p exactly 0 for every OTHER edge of the check,
 * whose output is then log 1 = 0: an edge whose exclusive set holds an a == 1 edge outputs exactly 0 (its sign
 * bit as any other output's).  (Pushes and a join with such a suffix keep D == S exactly, but the fma join with
 * such a prefix only to an ulp, which several zeros per check — erasures, quantized LLRs — add up to a flipped
 * hard decision: tests/golden/bp_zeros.npz.)  The rule is PER CODEWORD (fixz, round 6): it applies to a codeword
 * whose LLRs hold an exact zero (+-0) — the source of s = +-0 — for all its iterations, and not at all to the
 * others, where an a == 1 edge (an exact cancellation, or |s| so small that exp2 rounds to 1) keeps the plain
 * (D, S) outputs, within 2^-23 of 0; every GPU kernel applies the same rule (csrc/common.h).
 * Messages in LOG2 UNITS, as the GPU kernels keep them (ldpc-sims_amd/csrc/common.h): s2 = fma(L, log2 e, sum2),
 * a = exp2(-|s2|), the check output log2(S/D) clamped to [0, cmax2] with cmax2 = min(fp32(clamp * log2 e), 24 =
 * fp32(log2 RMAX)), z = fma(sum2, fp32(ln 2 / 2), 0.5 * L).  The trace reports messages in natural units (x ln 2). */
#define LOG2E_F32 1.44269502f      /* fp32(log2 e) = 0x1.715476p+0 */
#define HALF_LN2_F32 0.346573591f  /* fp32(ln 2 / 2) = 0x1.62e430p-2 */
#define LN2_F32 0.693147182f       /* fp32(ln 2) */
#define CEIL_LOG2_F32 24.0f        /* fp32(log2 16777215) */
static void cn_stable_f32(int d, const float* sa /* signed a per edge */, float cmax2, float* out,
                          float* sufD, float* sufS, int fixz) {
    if (d == 0) return;  /* an empty check (all-zero row of H) has no edges */
    if (d == 1) {  /* empty product = 1 -> the p clamp: S/D = 1/0 -> the ceiling */
        out[0] = cmax2;
        return;
    }
    uint32_t sg = 0;
    int n1 = 0;  /* edges with a == 1 */
    for (int t = 0; t < d; ++t) {
        sg ^= f2u(sa[t]);
        n1 += fixz && fabsf(sa[t]) == 1.0f;
    }
    sufD[d - 1] = fabsf(sa[d - 1]);
    sufS[d - 1] = 1.0f;
    for (int t = d - 2; t >= 1; --t) {
        const float a = fabsf(sa[t]);
        sufD[t] = fmaf(a, sufS[t + 1], sufD[t + 1]);
        sufS[t] = fmaf(a, sufD[t + 1], sufS[t + 1]);
    }
    float pD = 0.0f, pS = 1.0f;
    for (int t = 0; t < d; ++t) {
        float D, S;
        if (t == 0) { D = sufD[1]; S = sufS[1]; }
        else if (t == d - 1) { D = pD; S = pS; }
        else { D = fmaf(pD, sufS[t + 1], pS * sufD[t + 1]); S = fmaf(pD, sufD[t + 1], pS * sufS[t + 1]); }
        float y = log2f(S / D);   /* D == 0 (every other a underflowed): +inf -> the ceiling */
        if (!(y >= 0.0f)) y = 0.0f;  /* S >= D: a ratio rounded below 1 is log 1 */
        if (y > cmax2) y = cmax2;
        if (n1 - (fabsf(sa[t]) == 1.0f) > 0) y = 0.0f;  /* another edge has a == 1: the reference's p = 0 */
        out[t] = u2f(f2u(y) | ((sg ^ f2u(sa[t])) & 0x80000000u));
        const float a = fabsf(sa[t]);
        const float nD = fmaf(a, pS, pD), nS = fmaf(a, pD, pS);
        pD = nD;
        pS = nS;
    }
}

/* early stop (not in the reference): after iteration it >= 1, stop when the final layer's decisions
 * z = 0.5*(L + sum x) (bp.py:36-39,51) satisfy every check; returns the iterations run. */
static int sp_f32_one(const graph_t* g, const float* llr, int iters, float clamp, float* x, float* v2c,
                      float* p1_out, float* z_out, uint8_t* bits_out, float* trace, int64_t trace_stride,
                      int early_stop, uint8_t* hb, const wts_t* w, int stable, float* sufD, float* sufS) {
    const int E = g->E;
    int used = iters;
    const float c2 = clamp * LOG2E_F32, cmax2 = c2 < CEIL_LOG2_F32 ? c2 : CEIL_LOG2_F32;
    int fixz = 0;  /* an exact-zero LLR: the a == 1 rule's codewords (cn_stable_f32) */
    for (int v = 0; v < g->n; ++v) fixz |= llr[v] == 0.0f;
    for (int e = 0; e < E; ++e) x[e] = 0.0f;
    for (int it = 0; it < iters; ++it) {
        if (early_stop && it > 0) {
            for (int v = 0; v < g->n; ++v) {
                float S = 0.0f;
                for (int u = g->var_ptr[v]; u < g->var_ptr[v + 1]; ++u) S += x[g->var_edges[u]];
                const float zv = stable ? fmaf(S, HALF_LN2_F32, 0.5f * -llr[v]) : 0.5f * (-llr[v] + S);
                hb[v] = (uint8_t)(zv <= ZTHR_F32);
            }
            if (syndrome_ok(g, hb)) { used = it; break; }
        }
        /* VC + tanh: v2c at check-order ids */
        for (int v = 0; v < g->n; ++v) {
            const int a = g->var_ptr[v], b = g->var_ptr[v + 1], d = b - a;
            const float L = -llr[v];
            const float* wv = w && w->vn ? (const float*)w->vn + it * w->W + w->wofs[v] : NULL;
            const float Lw = w && w->lw ? ((const float*)w->lw)[(int64_t)it * g->n + v] * L : L;
            if (stable && !wv) {
                /* exclusive sums in O(d), the GPU kernels' order: suffix Q_t = x_t + ... + x_{d-1} (right to left),
                 * prefix P_t = x_0 + ... + x_{t-1} (left to right), S_0 = Q_1, S_{d-1} = P_{d-1}, S_t = P_t + Q_{t+1} */
                float* Q = sufD;  /* scratch, >= d entries */
                if (d >= 2) Q[d - 1] = x[g->var_edges[b - 1]];
                for (int t = d - 2; t >= 1; --t) Q[t] = Q[t + 1] + x[g->var_edges[a + t]];
                float P = 0.0f;
                for (int t = 0; t < d; ++t) {
                    const float xt = x[g->var_edges[a + t]];
                    const float S = d == 1 ? 0.0f : t == 0 ? Q[1] : t == d - 1 ? P : P + Q[t + 1];
                    P = t == 0 ? xt : P + xt;
                    const float sv = fmaf(Lw, LOG2E_F32, S);  /* log2 units */
                    v2c[g->var_edges[a + t]] = copysignf(exp2f(-fabsf(sv)), sv);
                }
                continue;
            }
            for (int t = a; t < b; ++t) {
                float S = 0.0f;
                if (stable) {  /* weighted: the O(d) association per target, sources before t left to right plus
                                  sources after t right to left (GPU k_vn_spw) */
                    float P = 0.0f, Q = 0.0f;
                    int hp = 0, hq = 0;
                    for (int u = b - 1; u > t; --u) {
                        const float y = wv[(t - a) * d + (u - a)] * x[g->var_edges[u]];
                        Q = hq ? Q + y : y;
                        hq = 1;
                    }
                    for (int u = a; u < t; ++u) {
                        const float y = wv[(t - a) * d + (u - a)] * x[g->var_edges[u]];
                        P = hp ? P + y : y;
                        hp = 1;
                    }
                    S = hp ? (hq ? P + Q : P) : (hq ? Q : 0.0f);
                } else {
                    for (int u = a; u < b; ++u)
                        if (u != t) S += wv ? wv[(t - a) * d + (u - a)] * x[g->var_edges[u]] : x[g->var_edges[u]];
                }
                if (stable) {  /* signed a = copysign(exp(-|s|), s), s = 2 * the reference's tanh argument */
                    const float sv = fmaf(Lw, LOG2E_F32, S);  /* log2 units */
                    v2c[g->var_edges[t]] = copysignf(exp2f(-fabsf(sv)), sv);
                } else {
                    v2c[g->var_edges[t]] = tanhf(0.5f * (Lw + S));
                }
            }
        }
        /* CV */
        for (int c = 0; c < g->m && stable; ++c) {
            const int a = g->row_ptr[c], b = g->row_ptr[c + 1];
            cn_stable_f32(b - a, v2c + a, cmax2, x + a, sufD, sufS, fixz);
        }
        for (int c = 0; c < g->m && !stable; ++c) {
            const int a = g->row_ptr[c], b = g->row_ptr[c + 1];
            for (int e = a; e < b; ++e) {
                float p = 1.0f;
                for (int u = a; u < b; ++u)
                    if (u != e) p *= v2c[u];
                if (p > PMAX_F32) p = PMAX_F32;
                if (p < -PMAX_F32) p = -PMAX_F32;
                float y = logf((1.0f + p) / (1.0f - p));
                if (y > clamp) y = clamp;
                if (y < -clamp) y = -clamp;
                x[e] = y;
            }
        }
        if (trace && stable)
            for (int e = 0; e < E; ++e) trace[(int64_t)it * trace_stride + e] = x[e] * LN2_F32;
        else if (trace)
            memcpy(trace + (int64_t)it * trace_stride, x, sizeof(float) * E);
    }
    for (int v = 0; v < g->n; ++v) {
        float S = 0.0f;
        const float* fw = w && w->fin ? (const float*)w->fin : NULL;
        for (int u = g->var_ptr[v]; u < g->var_ptr[v + 1]; ++u) S += fw ? fw[u] * x[g->var_edges[u]] : x[g->var_edges[u]];
        const float Lf = w && w->flw ? ((const float*)w->flw)[v] * -llr[v] : -llr[v];
        const float z = stable ? fmaf(S, HALF_LN2_F32, 0.5f * Lf) : 0.5f * (Lf + S);
        if (z_out) z_out[v] = z;
        if (p1_out) p1_out[v] = 1.0f - 1.0f / (1.0f + expf(-z));
        if (bits_out) bits_out[v] = (uint8_t)(z <= ZTHR_F32);
    }
    return used;
}

/* tanh sum-product, fp64: the reference module after .double() (pmax = PMAX_F64).  oracle_sp_f64_pmax passes
 * the fp32 module's bound (float)(1-1e-7) instead: fp64 arithmetic with the fp32 module's p-clamp ceiling
 * log(16777215), the target of the fp32 kernels' soft outputs when a caller's clamp exceeds 16.6355. */
static void sp_f64_one(const graph_t* g, const double* llr, int iters, double clamp, double pmax, double* x,
                       double* v2c, double* p1_out, double* z_out, uint8_t* bits_out, const wts_t* w) {
    const int E = g->E;
    for (int e = 0; e < E; ++e) x[e] = 0.0;
    for (int it = 0; it < iters; ++it) {
        for (int v = 0; v < g->n; ++v) {
            const int a = g->var_ptr[v], b = g->var_ptr[v + 1], d = b - a;
            const double L = -llr[v];
            const double* wv = w && w->vn ? (const double*)w->vn + it * w->W + w->wofs[v] : NULL;
            const double Lw = w && w->lw ? ((const double*)w->lw)[(int64_t)it * g->n + v] * L : L;
            for (int t = a; t < b; ++t) {
                double S = 0.0;
                for (int u = a; u < b; ++u)
                    if (u != t) S += wv ? wv[(t - a) * d + (u - a)] * x[g->var_edges[u]] : x[g->var_edges[u]];
                v2c[g->var_edges[t]] = tanh(0.5 * (Lw + S));
            }
        }
        for (int c = 0; c < g->m; ++c) {
            const int a = g->row_ptr[c], b = g->row_ptr[c + 1];
            for (int e = a; e < b; ++e) {
                double p = 1.0;
                for (int u = a; u < b; ++u)
                    if (u != e) p *= v2c[u];
                if (p > pmax) p = pmax;
                if (p < -pmax) p = -pmax;
                double y = log((1.0 + p) / (1.0 - p));
                if (y > clamp) y = clamp;
                if (y < -clamp) y = -clamp;
                x[e] = y;
            }
        }
    }
    for (int v = 0; v < g->n; ++v) {
        double S = 0.0;
        const double* fw = w && w->fin ? (const double*)w->fin : NULL;
        for (int u = g->var_ptr[v]; u < g->var_ptr[v + 1]; ++u) S += fw ? fw[u] * x[g->var_edges[u]] : x[g->var_edges[u]];
        const double Lf = w && w->flw ? ((const double*)w->flw)[v] * -llr[v] : -llr[v];
        const double z = 0.5 * (Lf + S);
        if (z_out) z_out[v] = z;
        if (p1_out) p1_out[v] = 1.0 - 1.0 / (1.0 + exp(-z));
        if (bits_out) bits_out[v] = (uint8_t)(z < ZTHR_F64);
    }
}

static int syndrome_ok(const graph_t* g, const uint8_t* bits) {
    for (int c = 0; c < g->m; ++c) {
        int par = 0;
        for (int e = g->row_ptr[c]; e < g->row_ptr[c + 1]; ++e) par ^= bits[g->col_idx[e]];
        if (par) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* min-sum, fp32 (specification above; no reference counterpart)                               */
static int ms_f32_one(const graph_t* g, const float* llr, int iters, float clamp, float alpha, float beta,
                      int early_stop, float* c2v, float* app, uint8_t* hb, float* p1_out, float* z_out,
                      uint8_t* bits_out) {
    const int E = g->E, n = g->n;
    for (int e = 0; e < E; ++e) c2v[e] = 0.0f;
    for (int v = 0; v < n; ++v) {
        float s = -llr[v];
        for (int u = g->var_ptr[v]; u < g->var_ptr[v + 1]; ++u) s += c2v[g->var_edges[u]];
        app[v] = s;
    }
    int used = 0;
    for (int it = 0; it < iters; ++it) {
        for (int c = 0; c < g->m; ++c) {
            const int a = g->row_ptr[c], b = g->row_ptr[c + 1];
            float min1 = INFINITY, min2 = INFINITY;
            int idx = -1;
            uint32_t sgn = 0;
            for (int e = a; e < b; ++e) {
                const float t = app[g->col_idx[e]] - c2v[e];
                const float m = fabsf(t);
                sgn ^= f2u(t);
                if (m < min1) { min2 = min1; min1 = m; idx = e; }
                else if (m < min2) { min2 = m; }
            }
            sgn &= 0x80000000u;
            for (int e = a; e < b; ++e) {
                const float t = app[g->col_idx[e]] - c2v[e]; /* recomputed from the OLD c2v[e] */
                float mag = (e == idx) ? min2 : min1;
                mag = alpha * mag;
                mag = fmaxf(mag - beta, 0.0f);
                mag = fminf(mag, clamp);
                c2v[e] = u2f(f2u(mag) | ((sgn ^ f2u(t)) & 0x80000000u));
            }
        }
        for (int v = 0; v < n; ++v) {
            float s = -llr[v];
            for (int u = g->var_ptr[v]; u < g->var_ptr[v + 1]; ++u) s += c2v[g->var_edges[u]];
            app[v] = s;
        }
        used = it + 1;
        if (early_stop) {
            for (int v = 0; v < n; ++v) hb[v] = (uint8_t)(0.5f * app[v] <= ZTHR_F32);
            if (syndrome_ok(g, hb)) break;
        }
    }
    for (int v = 0; v < n; ++v) {
        const float z = 0.5f * app[v];
        if (z_out) z_out[v] = z;
        if (p1_out) p1_out[v] = 1.0f - 1.0f / (1.0f + expf(-z));
        if (bits_out) bits_out[v] = (uint8_t)(z <= ZTHR_F32);
    }
    return used;
}

/* ------------------------------------------------------------------------------------------ */
/* quantized (integer) offset min-sum: llr already quantized to int8 in [-qmax, qmax]           */
static inline int sat(int x, int lim) { return x > lim ? lim : (x < -lim ? -lim : x); }

static int qms_one(const graph_t* g, const int8_t* qllr, int iters, int qmax, int app_max, int beta,
                   int early_stop, int8_t* c2v, int16_t* app, uint8_t* hb, int16_t* app_out, uint8_t* bits_out) {
    const int E = g->E, n = g->n;
    for (int e = 0; e < E; ++e) c2v[e] = 0;
    for (int v = 0; v < n; ++v) app[v] = (int16_t)sat(-(int)qllr[v], app_max);
    int used = 0;
    for (int it = 0; it < iters; ++it) {
        for (int c = 0; c < g->m; ++c) {
            const int a = g->row_ptr[c], b = g->row_ptr[c + 1];
            int min1 = 1 << 30, min2 = 1 << 30, idx = -1, sgn = 0;
            for (int e = a; e < b; ++e) {
                const int t = sat((int)app[g->col_idx[e]] - (int)c2v[e], qmax);
                const int m = t < 0 ? -t : t;
                sgn ^= (t < 0);
                if (m < min1) { min2 = min1; min1 = m; idx = e; }
                else if (m < min2) { min2 = m; }
            }
            for (int e = a; e < b; ++e) {
                const int t = sat((int)app[g->col_idx[e]] - (int)c2v[e], qmax);
                int mag = (e == idx) ? min2 : min1;
                mag = mag - beta;
                if (mag < 0) mag = 0;
                if (mag > qmax) mag = qmax;
                c2v[e] = (int8_t)((sgn ^ (t < 0)) ? -mag : mag);
            }
        }
        for (int v = 0; v < n; ++v) {
            int s = -(int)qllr[v];
            for (int u = g->var_ptr[v]; u < g->var_ptr[v + 1]; ++u) s += c2v[g->var_edges[u]];
            app[v] = (int16_t)sat(s, app_max);
        }
        used = it + 1;
        if (early_stop) {
            for (int v = 0; v < n; ++v) hb[v] = (uint8_t)(app[v] < 0);
            if (syndrome_ok(g, hb)) break;
        }
    }
    for (int v = 0; v < n; ++v) {
        if (app_out) app_out[v] = app[v];
        if (bits_out) bits_out[v] = (uint8_t)(app[v] < 0);
    }
    return used;
}

/* ------------------------------------------------------------------------------------------ */
/* exported entry points (ctypes).  All arrays row-major [B][n]; outputs may be NULL.             */
#define GRAPH_ARGS int m, int n, int E, const int32_t *row_ptr, const int32_t *col_idx, \
                   const int32_t *var_ptr, const int32_t *var_edges
#define MAKE_GRAPH graph_t g = {m, n, E, row_ptr, col_idx, var_ptr, var_edges}
#define WEIGHT_ARGS const void *w_vn, const void *w_lw, const void *w_fin, const void *w_flw

/* fills wt (and allocates wofs) when any weight array is given; returns the pointer to pass, or NULL */
static const wts_t* make_wts(const graph_t* g, wts_t* wt, WEIGHT_ARGS) {
    if (!w_vn && !w_lw && !w_fin && !w_flw) return NULL;
    int64_t* wofs = (int64_t*)malloc(sizeof(int64_t) * ((size_t)g->n + 1));
    wofs[0] = 0;
    for (int v = 0; v < g->n; ++v) {
        const int64_t d = g->var_ptr[v + 1] - g->var_ptr[v];
        wofs[v + 1] = wofs[v] + d * d;
    }
    wt->vn = w_vn;
    wt->lw = w_lw;
    wt->fin = w_fin;
    wt->flw = w_flw;
    wt->wofs = wofs;
    wt->W = wofs[g->n];
    return wt;
}

/* stable = 0: the reference's fp32 operations (tanh, masked product, log((1+p)/(1-p))); 1: the (D, S) form
 * of cn_stable_f32, the specification the GPU tanh-SP kernels follow. */
int oracle_sp_f32(GRAPH_ARGS, const float* llr, int64_t B, int iters, float clamp, float* p1, float* z,
                  uint8_t* bits, float* trace /* [iters][B][E] or NULL */, int early_stop, int32_t* iters_used,
                  WEIGHT_ARGS, int stable) {
    MAKE_GRAPH;
    wts_t wt;
    const wts_t* w = make_wts(&g, &wt, w_vn, w_lw, w_fin, w_flw);
    if (w && early_stop) { free((void*)wt.wofs); return -1; }
#pragma omp parallel
    {
        float* x = (float*)malloc(sizeof(float) * (size_t)E);
        float* v2c = (float*)malloc(sizeof(float) * (size_t)E);
        float* suf = (float*)malloc(sizeof(float) * 2 * (size_t)E);
        uint8_t* hb = (uint8_t*)malloc((size_t)n);
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < B; ++i) {
            int u = sp_f32_one(&g, llr + i * n, iters, clamp, x, v2c, p1 ? p1 + i * n : NULL, z ? z + i * n : NULL,
                               bits ? bits + i * n : NULL, trace ? trace + i * E : NULL, B * (int64_t)E, early_stop, hb, w,
                               stable, suf, suf + E);
            if (iters_used) iters_used[i] = u;
        }
        free(suf);
        free(x);
        free(v2c);
        free(hb);
    }
    if (w) free((void*)wt.wofs);
    return 0;
}

int oracle_sp_f64_pmax(GRAPH_ARGS, const double* llr, int64_t B, int iters, double clamp, double pmax, double* p1,
                       double* z, uint8_t* bits, WEIGHT_ARGS) {
    MAKE_GRAPH;
    wts_t wt;
    const wts_t* w = make_wts(&g, &wt, w_vn, w_lw, w_fin, w_flw);
#pragma omp parallel
    {
        double* x = (double*)malloc(sizeof(double) * (size_t)E);
        double* v2c = (double*)malloc(sizeof(double) * (size_t)E);
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < B; ++i)
            sp_f64_one(&g, llr + i * n, iters, clamp, pmax, x, v2c, p1 ? p1 + i * n : NULL, z ? z + i * n : NULL,
                       bits ? bits + i * n : NULL, w);
        free(x);
        free(v2c);
    }
    if (w) free((void*)wt.wofs);
    return 0;
}

int oracle_sp_f64(GRAPH_ARGS, const double* llr, int64_t B, int iters, double clamp, double* p1, double* z,
                  uint8_t* bits, WEIGHT_ARGS) {
    return oracle_sp_f64_pmax(m, n, E, row_ptr, col_idx, var_ptr, var_edges, llr, B, iters, clamp, PMAX_F64, p1, z,
                              bits, w_vn, w_lw, w_fin, w_flw);
}

int oracle_ms_f32(GRAPH_ARGS, const float* llr, int64_t B, int iters, float clamp, float alpha, float beta,
                  int early_stop, float* p1, float* z, uint8_t* bits, int32_t* iters_used) {
    MAKE_GRAPH;
#pragma omp parallel
    {
        float* c2v = (float*)malloc(sizeof(float) * (size_t)E);
        float* app = (float*)malloc(sizeof(float) * (size_t)n);
        uint8_t* hb = (uint8_t*)malloc((size_t)n);
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < B; ++i) {
            int u = ms_f32_one(&g, llr + i * n, iters, clamp, alpha, beta, early_stop, c2v, app, hb,
                               p1 ? p1 + i * n : NULL, z ? z + i * n : NULL, bits ? bits + i * n : NULL);
            if (iters_used) iters_used[i] = u;
        }
        free(c2v);
        free(app);
        free(hb);
    }
    return 0;
}

int oracle_qms(GRAPH_ARGS, const int8_t* qllr, int64_t B, int iters, int qmax, int app_max, int beta,
               int early_stop, int16_t* app_out, uint8_t* bits, int32_t* iters_used) {
    MAKE_GRAPH;
#pragma omp parallel
    {
        int8_t* c2v = (int8_t*)malloc((size_t)E);
        int16_t* app = (int16_t*)malloc(sizeof(int16_t) * (size_t)n);
        uint8_t* hb = (uint8_t*)malloc((size_t)n);
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < B; ++i) {
            int u = qms_one(&g, qllr + i * n, iters, qmax, app_max, beta, early_stop, c2v, app, hb,
                            app_out ? app_out + i * n : NULL, bits ? bits + i * n : NULL);
            if (iters_used) iters_used[i] = u;
        }
        free(c2v);
        free(app);
        free(hb);
    }
    return 0;
}

int oracle_num_threads(void) {
    int t = 1;
#pragma omp parallel
    {
#pragma omp master
        {
#ifdef _OPENMP
            extern int omp_get_num_threads(void);
            t = omp_get_num_threads();
#endif
        }
    }
    return t;
}
