// generic.hip — CSR flooding BP kernels for ANY parity-check matrix (gfx950).
//
// Data layout in HBM (codeword-interleaved, "edge-major"): every per-edge or per-variable quantity is a
// row of `ldb` floats, one column per codeword, ldb = B rounded up to 64:
//     L[n][ldb]      = -llr                         (P0/P1 convention, bp/bp.py:47 negates inside)
//     v2c[E][ldb]    variable->check message at the reference's CHECK-ORDER edge id (bp/masking.py:84-88)
//     c2v[E][ldb]    check->variable message (the reference's x tensor, bp/bp.py:46-47)
// A workgroup owns one check (or one variable) for 256 codewords, so the graph lookups
// (row_ptr/var_ptr/var_edges at blockIdx.y) are wave-uniform scalar loads and every message access is a
// fully coalesced 1 KiB row segment.  This is the reference's own two-array flooding dataflow
// (SURVEY.md §8(d)): per iteration each kernel streams its messages through HBM once, so it is
// HBM-bound by construction: bytes/cw/iter = 4*E*s + n*s.
//
//   tanh-SP  k_vn_sp : v2c = tanh(0.5*(L + sum_{c'!=c} c2v))           bp_vc.py:16-27 + bp.py:29
//            k_cn_sp : c2v = clamp(log((1+p)/(1-p)), +-clamp), p = clamp(prod_{v'!=v} v2c, +-(1-1e-7))
//                                                                        bp_cv.py:22-50 + bp.py:47
//   min-sum  k_vn_ms / k_cn_ms                                          (oracle/ldpc_oracle.c spec)
//   k_final  : z = 0.5*(L + sum c2v), bits = np.round(1-sigmoid(z)), p1 = 1-sigmoid(z)   bp.py:51
//
// Exclusive sums/products use the prefix-then-continue form, which performs exactly the sequential
// operations of the reference's masked reductions ("skip self, ascending order").
#include "common.h"

namespace ldpc {

constexpr int kTB = 256;

template <typename T>
__global__ __launch_bounds__(256) void k_load_llr(const T* __restrict__ llr, T* __restrict__ L, int64_t B, int n,
                                                  int64_t ldb) {
    __shared__ T tile[64][65];
    const int64_t cw0 = (int64_t)blockIdx.x * 64;
    const int v0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int64_t cw = cw0 + r;
        const int v = v0 + tx;
        if (cw < B && v < n) tile[r][tx] = -llr[cw * n + v];
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int v = v0 + r;
        const int64_t cw = cw0 + tx;
        if (v < n && cw < B) L[(int64_t)v * ldb + cw] = tile[tx][r];
    }
}

// V codewords per thread: every message access is a 16-byte-per-lane load/store (a wave moves 1 KiB per
// instruction).  V = 4 floats (2 doubles) for small degrees; fewer when MAXD*V values would not fit.
template <typename T, int MAXD>
struct VW {
    static constexpr int v16 = 16 / (int)sizeof(T);
    static constexpr int value = (MAXD <= 8) ? v16 : (MAXD <= 16 ? (v16 >= 2 ? v16 / 2 : 1) : 1);
};

template <typename T, int V>
struct Vec {
    T x[V];
};
template <typename T, int V>
__device__ __forceinline__ Vec<T, V> vload(const T* p) {
    Vec<T, V> r;
    if constexpr (V * sizeof(T) == 16) {
        using U = __attribute__((ext_vector_type(4))) float;
        const U u = *reinterpret_cast<const U*>(p);
        __builtin_memcpy(r.x, &u, 16);
    } else if constexpr (V * sizeof(T) == 8) {
        using U = __attribute__((ext_vector_type(2))) float;
        const U u = *reinterpret_cast<const U*>(p);
        __builtin_memcpy(r.x, &u, 8);
    } else {
#pragma unroll
        for (int i = 0; i < V; ++i) r.x[i] = p[i];
    }
    return r;
}
template <typename T, int V>
__device__ __forceinline__ void vstore(T* p, const Vec<T, V>& r) {
    if constexpr (V * sizeof(T) == 16) {
        using U = __attribute__((ext_vector_type(4))) float;
        U u;
        __builtin_memcpy(&u, r.x, 16);
        *reinterpret_cast<U*>(p) = u;
    } else if constexpr (V * sizeof(T) == 8) {
        using U = __attribute__((ext_vector_type(2))) float;
        U u;
        __builtin_memcpy(&u, r.x, 8);
        *reinterpret_cast<U*>(p) = u;
    } else {
#pragma unroll
        for (int i = 0; i < V; ++i) p[i] = r.x[i];
    }
}

// Loads are issued for all MAXD slots with the edge index clamped to the last valid one (harmless
// duplicate reads): a wave-uniform `if (k < d)` around each load makes hipcc branch around it and
// drain vmcnt per load (cdna_hip_programming.md §5, load-reduce trap (c)).

template <typename T, int MAXD>
__global__ __launch_bounds__(256) void k_vn_sp(const int32_t* __restrict__ var_ptr, const int32_t* __restrict__ var_edges,
                                               const T* __restrict__ L, const T* __restrict__ c2v, T* __restrict__ v2c,
                                               int64_t B, int64_t ldb, int first) {
    constexpr int V = VW<T, MAXD>::value;
    const int v = blockIdx.y;
    const int64_t cw = ((int64_t)blockIdx.x * kTB + threadIdx.x) * V;
    if (cw >= B) return;
    const int a = var_ptr[v];
    const int d = var_ptr[v + 1] - a;
    if (d == 0) return;  // an all-zero column of H has no messages (k_final still decides it)
    const Vec<T, V> Lv = vload<T, V>(L + (int64_t)v * ldb + cw);
    Vec<T, V> x[MAXD];
    int64_t off[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        off[k] = (int64_t)var_edges[a + (k < d ? k : d - 1)] * ldb + cw;
        if (first) {
#pragma unroll
            for (int i = 0; i < V; ++i) x[k].x[i] = T(0);
        } else {
            x[k] = vload<T, V>(c2v + off[k]);
        }
    }
    Vec<T, V> P;
#pragma unroll
    for (int i = 0; i < V; ++i) P.x[i] = T(0);
#pragma unroll
    for (int t = 0; t < MAXD; ++t)
        if (t < d) {
            Vec<T, V> o;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                T S = P.x[i];
#pragma unroll
                for (int u = t + 1; u < MAXD; ++u)
                    if (u < d) S += x[u].x[i];
                o.x[i] = Num<T>::tanh_(T(0.5) * (Lv.x[i] + S));
                P.x[i] += x[t].x[i];
            }
            vstore<T, V>(v2c + off[t], o);
        }
}

template <typename T, int MAXD>
__global__ __launch_bounds__(256) void k_cn_sp(const int32_t* __restrict__ row_ptr, const T* __restrict__ v2c,
                                               T* __restrict__ c2v, int64_t B, int64_t ldb, T clamp) {
    constexpr int V = VW<T, MAXD>::value;
    const int c = blockIdx.y;
    const int64_t cw = ((int64_t)blockIdx.x * kTB + threadIdx.x) * V;
    if (cw >= B) return;
    const int a = row_ptr[c];
    const int d = row_ptr[c + 1] - a;
    if (d == 0) return;  // an empty check carries no messages
    Vec<T, V> t[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) t[k] = vload<T, V>(v2c + (int64_t)(a + (k < d ? k : d - 1)) * ldb + cw);
    Vec<T, V> Q;
#pragma unroll
    for (int i = 0; i < V; ++i) Q.x[i] = T(1);
#pragma unroll
    for (int e = 0; e < MAXD; ++e)
        if (e < d) {
            Vec<T, V> o;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                T p = Q.x[i];
#pragma unroll
                for (int u = e + 1; u < MAXD; ++u)
                    if (u < d) p *= t[u].x[i];
                if (p > Num<T>::pmax) p = Num<T>::pmax;
                if (p < -Num<T>::pmax) p = -Num<T>::pmax;
                T y = Num<T>::log_((T(1) + p) / (T(1) - p));
                if (y > clamp) y = clamp;
                if (y < -clamp) y = -clamp;
                o.x[i] = y;
                Q.x[i] *= t[e].x[i];
            }
            vstore<T, V>(c2v + (int64_t)(a + e) * ldb + cw, o);
        }
}

template <int MAXD>
__global__ __launch_bounds__(256) void k_vn_ms(const int32_t* __restrict__ var_ptr, const int32_t* __restrict__ var_edges,
                                               const float* __restrict__ L, const float* __restrict__ c2v,
                                               float* __restrict__ v2c, int64_t B, int64_t ldb, int first) {
    constexpr int V = VW<float, MAXD>::value;
    const int v = blockIdx.y;
    const int64_t cw = ((int64_t)blockIdx.x * kTB + threadIdx.x) * V;
    if (cw >= B) return;
    const int a = var_ptr[v];
    const int d = var_ptr[v + 1] - a;
    if (d == 0) return;
    Vec<float, V> app = vload<float, V>(L + (int64_t)v * ldb + cw);
    Vec<float, V> x[MAXD];
    int64_t off[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        off[k] = (int64_t)var_edges[a + (k < d ? k : d - 1)] * ldb + cw;
        if (first) {
#pragma unroll
            for (int i = 0; i < V; ++i) x[k].x[i] = 0.0f;
        } else {
            x[k] = vload<float, V>(c2v + off[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < MAXD; ++k)
        if (k < d) {
#pragma unroll
            for (int i = 0; i < V; ++i) app.x[i] += x[k].x[i];
        }
#pragma unroll
    for (int k = 0; k < MAXD; ++k)
        if (k < d) {
            Vec<float, V> o;
#pragma unroll
            for (int i = 0; i < V; ++i) o.x[i] = app.x[i] - x[k].x[i];
            vstore<float, V>(v2c + off[k], o);
        }
}

template <int MAXD>
__global__ __launch_bounds__(256) void k_cn_ms(const int32_t* __restrict__ row_ptr, const float* __restrict__ v2c,
                                               float* __restrict__ c2v, int64_t B, int64_t ldb, float clamp,
                                               float alpha, float beta) {
    constexpr int V = VW<float, MAXD>::value;
    const int c = blockIdx.y;
    const int64_t cw = ((int64_t)blockIdx.x * kTB + threadIdx.x) * V;
    if (cw >= B) return;
    const int a = row_ptr[c];
    const int d = row_ptr[c + 1] - a;
    if (d == 0) return;
    Vec<float, V> t[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) t[k] = vload<float, V>(v2c + (int64_t)(a + (k < d ? k : d - 1)) * ldb + cw);
#pragma unroll
    for (int i = 0; i < V; ++i) {
        float min1 = __builtin_inff(), min2 = __builtin_inff();
        int idx = -1;
        uint32_t sgn = 0;
#pragma unroll
        for (int k = 0; k < MAXD; ++k)
            if (k < d) {
                const float m = fabsf(t[k].x[i]);
                sgn ^= f2u(t[k].x[i]);
                if (m < min1) {
                    min2 = min1;
                    min1 = m;
                    idx = k;
                } else if (m < min2) {
                    min2 = m;
                }
            }
        const float mag1 = ms_mag(min1, alpha, beta, clamp);
        const float mag2 = ms_mag(min2, alpha, beta, clamp);
#pragma unroll
        for (int k = 0; k < MAXD; ++k)
            if (k < d) {
                const float mag = (k == idx) ? mag2 : mag1;
                t[k].x[i] = u2f(f2u(mag) | ((sgn ^ f2u(t[k].x[i])) & 0x80000000u));
            }
    }
#pragma unroll
    for (int k = 0; k < MAXD; ++k)
        if (k < d) vstore<float, V>(c2v + (int64_t)(a + k) * ldb + cw, t[k]);
}

// Final VC + sigmoid + hard decision (bp/bp.py:36-39,51; ofdm_functions.py:161), transposed back to
// the caller's [B][n] layout through an LDS tile.
template <typename T, int MAXD, bool MS>
__global__ __launch_bounds__(256) void k_final(const int32_t* __restrict__ var_ptr, const int32_t* __restrict__ var_edges,
                                               const T* __restrict__ L, const T* __restrict__ c2v, int64_t B,
                                               int64_t ldb, int n, uint8_t* __restrict__ bits, T* __restrict__ soft,
                                               int soft_z) {
    __shared__ T zt[64][65];
    const int64_t cw0 = (int64_t)blockIdx.x * 64;
    const int v0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int vr = ty; vr < 64; vr += 4) {
        const int v = v0 + vr;
        const int64_t cw = cw0 + tx;
        if (v < n && cw < B) {
            const int a = var_ptr[v];
            const int d = var_ptr[v + 1] - a;
            const T Lv = L[(int64_t)v * ldb + cw];
            T z;
            if (MS) {
                T app = Lv;
                for (int k = 0; k < d; ++k) app += c2v[(int64_t)var_edges[a + k] * ldb + cw];
                z = T(0.5) * app;
            } else {
                T S = T(0);
                for (int k = 0; k < d; ++k) S += c2v[(int64_t)var_edges[a + k] * ldb + cw];
                z = T(0.5) * (Lv + S);
            }
            zt[vr][tx] = z;
        }
    }
    __syncthreads();
    for (int cr = ty; cr < 64; cr += 4) {
        const int64_t cw = cw0 + cr;
        const int v = v0 + tx;
        if (v < n && cw < B) {
            const T z = zt[tx][cr];
            if (bits) bits[cw * n + v] = (uint8_t)Num<T>::bit(z);
            if (soft) soft[cw * n + v] = soft_z ? z : T(1) - T(1) / (T(1) + Num<T>::exp_(-z));
        }
    }
}

// ------------------------------------------------------------------------------------------------
static int pick_maxd(int d) {
    return d <= 4 ? 4 : d <= 8 ? 8 : d <= 12 ? 12 : d <= 16 ? 16 : d <= 20 ? 20 : d <= 24 ? 24 : d <= 32 ? 32 : -1;
}

template <typename T>
static int run_sp(const GenericArgs& g, const T* llr_dev, int64_t B, int iters, T clamp, uint8_t* bits, T* soft,
                  int soft_z, char* ws, hipStream_t st) {
    const int64_t ldb = (B + 63) / 64 * 64;
    T* L = (T*)ws;
    T* v2c = L + (int64_t)g.n * ldb;
    T* c2v = v2c + (int64_t)g.E * ldb;
    const dim3 tb(kTB);
    auto gxv = [B](int V) { return (unsigned)((B + (int64_t)kTB * V - 1) / ((int64_t)kTB * V)); };
    k_load_llr<T><<<dim3((unsigned)((B + 63) / 64), (g.n + 63) / 64), tb, 0, st>>>(llr_dev, L, B, g.n, ldb);
    const int dv = pick_maxd(g.max_dv), dc = pick_maxd(g.max_dc);
    if (dv < 0 || dc < 0) return set_error(LDPC_EUNSUPPORTED, "node degree > 32 not supported by generic kernels");
    for (int it = 0; it < iters; ++it) {
        const int first = (it == 0);
#define VN(D) k_vn_sp<T, D><<<dim3(gxv(VW<T, D>::value), g.n), tb, 0, st>>>(g.var_ptr, g.var_edges, L, c2v, v2c, B, ldb, first)
        switch (dv) { case 4: VN(4); break; case 8: VN(8); break; case 12: VN(12); break; case 16: VN(16); break; case 20: VN(20); break; case 24: VN(24); break; default: VN(32); }
#undef VN
#define CN(D) k_cn_sp<T, D><<<dim3(gxv(VW<T, D>::value), g.m), tb, 0, st>>>(g.row_ptr, v2c, c2v, B, ldb, clamp)
        switch (dc) { case 4: CN(4); break; case 8: CN(8); break; case 12: CN(12); break; case 16: CN(16); break; case 20: CN(20); break; case 24: CN(24); break; default: CN(32); }
#undef CN
    }
    if (iters == 0) (void)hipMemsetAsync(c2v, 0, sizeof(T) * (size_t)g.E * ldb, st);
    k_final<T, 32, false><<<dim3((unsigned)((B + 63) / 64), (g.n + 63) / 64), tb, 0, st>>>(
        g.var_ptr, g.var_edges, L, c2v, B, ldb, g.n, bits, soft, soft_z);
    return LDPC_OK;
}

static int run_ms(const GenericArgs& g, const float* llr_dev, int64_t B, int iters, float clamp, float alpha, float beta,
                  uint8_t* bits, float* soft, int soft_z, char* ws, hipStream_t st) {
    const int64_t ldb = (B + 63) / 64 * 64;
    float* L = (float*)ws;
    float* v2c = L + (int64_t)g.n * ldb;
    float* c2v = v2c + (int64_t)g.E * ldb;
    const dim3 tb(kTB);
    auto gxv = [B](int V) { return (unsigned)((B + (int64_t)kTB * V - 1) / ((int64_t)kTB * V)); };
    k_load_llr<float><<<dim3((unsigned)((B + 63) / 64), (g.n + 63) / 64), tb, 0, st>>>(llr_dev, L, B, g.n, ldb);
    const int dv = pick_maxd(g.max_dv), dc = pick_maxd(g.max_dc);
    if (dv < 0 || dc < 0) return set_error(LDPC_EUNSUPPORTED, "node degree > 32 not supported by generic kernels");
    for (int it = 0; it < iters; ++it) {
        const int first = (it == 0);
#define VN(D) k_vn_ms<D><<<dim3(gxv(VW<float, D>::value), g.n), tb, 0, st>>>(g.var_ptr, g.var_edges, L, c2v, v2c, B, ldb, first)
        switch (dv) { case 4: VN(4); break; case 8: VN(8); break; case 12: VN(12); break; case 16: VN(16); break; case 20: VN(20); break; case 24: VN(24); break; default: VN(32); }
#undef VN
#define CN(D) k_cn_ms<D><<<dim3(gxv(VW<float, D>::value), g.m), tb, 0, st>>>(g.row_ptr, v2c, c2v, B, ldb, clamp, alpha, beta)
        switch (dc) { case 4: CN(4); break; case 8: CN(8); break; case 12: CN(12); break; case 16: CN(16); break; case 20: CN(20); break; case 24: CN(24); break; default: CN(32); }
#undef CN
    }
    if (iters == 0) (void)hipMemsetAsync(c2v, 0, sizeof(float) * (size_t)g.E * ldb, st);
    k_final<float, 32, true><<<dim3((unsigned)((B + 63) / 64), (g.n + 63) / 64), tb, 0, st>>>(
        g.var_ptr, g.var_edges, L, c2v, B, ldb, g.n, bits, soft, soft_z);
    return LDPC_OK;
}

size_t generic_workspace(int n, int E, int64_t B, size_t elem) {
    const int64_t ldb = (B + 63) / 64 * 64;
    return elem * (size_t)ldb * ((size_t)n + 2 * (size_t)E);
}

int generic_decode(const GenericArgs& g, const void* llr_dev, int64_t B, const ldpc_params& p, uint8_t* bits,
                   void* soft, int32_t* iters_used, char* ws, hipStream_t st) {
    const int soft_z = (p.flags & LDPC_F_SOFT_Z) ? 1 : 0;
    if (p.flags & LDPC_F_EARLY_STOP)
        return set_error(LDPC_EUNSUPPORTED, "early stop is implemented by the QC kernels only");
    int rc;
    if (p.algo == LDPC_ALGO_TANH_SP) {
        if (p.flags & LDPC_F_F64)
            rc = run_sp<double>(g, (const double*)llr_dev, B, p.iters, (double)p.clamp, bits, (double*)soft, soft_z, ws, st);
        else
            rc = run_sp<float>(g, (const float*)llr_dev, B, p.iters, p.clamp, bits, (float*)soft, soft_z, ws, st);
    } else if (p.algo == LDPC_ALGO_MIN_SUM) {
        if (p.flags & LDPC_F_F64) return set_error(LDPC_EUNSUPPORTED, "min-sum is float32 only");
        rc = run_ms(g, (const float*)llr_dev, B, p.iters, p.clamp, p.alpha, p.beta, bits, (float*)soft, soft_z, ws, st);
    } else {
        return set_error(LDPC_EUNSUPPORTED, "algo %d not supported by the generic kernels", p.algo);
    }
    if (rc != LDPC_OK) return rc;
    if (iters_used) {
        // every codeword runs the fixed iteration count
        rc = fill_i32(iters_used, B, p.iters, st);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "generic kernel launch: %s", hipGetErrorString(e));
    return rc;
}

}  // namespace ldpc
