// generic_impl.h — CSR flooding BP kernels for ANY parity-check matrix (gfx950).  Included by generic.hip
// (entry points, chunking) and generic_run.hip, which is compiled once per (precision, algorithm, early
// stop) driver instantiation so the kernel templates build in parallel translation units.
//
// Data layout in HBM (codeword-interleaved, "edge-major"): every per-edge or per-variable quantity is a
// row of `ldb` floats, one column per codeword, ldb = B rounded up to 64:
//     L[n][ldb]      = -llr                         (P0/P1 convention, bp/bp.py:47 negates inside)
//     v2c[E][ldb]    variable->check message at the reference's CHECK-ORDER edge id (bp/masking.py:84-88)
//     c2v[E][ldb]    check->variable message (the reference's x tensor, bp/bp.py:46-47)
// A wave owns one check (or one variable) for 64*V codewords (tile_slot), so the graph lookups
// (row_ptr/var_ptr/var_edges) are wave-uniform scalar loads and every message access is a fully
// coalesced row segment of 256 B - 1 KiB.  This is the reference's own two-array flooding dataflow
// (SURVEY.md §8(d)): per iteration each kernel streams its messages through HBM once, so it is
// HBM-bound by construction: bytes/cw/iter = 4*E*s + n*s.
//
//   tanh-SP  k_vn_sp : v2c = tanh(0.5*(L + sum_{c'!=c} c2v))           bp_vc.py:16-27 + bp.py:29
//            k_cn_sp : c2v = clamp(log((1+p)/(1-p)), +-clamp), p = clamp(prod_{v'!=v} v2c, +-(1-1e-7))
//                                                                        bp_cv.py:22-50 + bp.py:47
//            fp32 evaluates this function in the (D, S) form with messages in log2 units (common.h): the VN
//            stores the signed a = copysign(exp2(-|s2|), s2) instead of tanh(s/2) with O(d) exclusive sums,
//            the CN forms each edge's exclusive set from prefix and suffix sets (O(d)) and outputs
//            log2(S/D); fp64 keeps the reference's operations.
//   min-sum  k_vn_ms / k_cn_ms                                          (oracle/ldpc_oracle.c spec)
//   k_final  : z = 0.5*(L + sum c2v), bits = np.round(1-sigmoid(z)), p1 = 1-sigmoid(z)   bp.py:51
//
// fp64 exclusive sums/products use the prefix-then-continue form, the sequential operations of the reference's
// masked reductions ("skip self, ascending order"); fp32 tanh-SP and min-sum follow the oracle's orders.
#pragma once
#include "common.h"

namespace ldpc {

constexpr int kTB = 256;

// [B][n] row-major -> [n][ldb] edge-major, times `scale`: -1 for the LLR (the reference decodes -llr, bp.py:47),
// +1 for initial c2v messages (n = E; fp32 tanh-SP: log2 e, its messages are in log2 units, common.h)
template <typename T>
__global__ __launch_bounds__(256) void k_load_llr(const T* __restrict__ llr, T* __restrict__ L, int64_t B, int n,
                                                  int64_t ldb, T scale) {
    __shared__ T tile[64][65];
    const int64_t cw0 = (int64_t)blockIdx.x * 64;
    const int v0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int64_t cw = cw0 + r;
        const int v = v0 + tx;
        if (cw < B && v < n) tile[r][tx] = llr[cw * n + v] * scale;
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

// Tile of a 256-thread workgroup: 2^tpl2 threads (tpl2 in 6..8, whole waves) per node, V codewords per
// thread, so 256 >> tpl2 nodes per workgroup.  The node index is wave-uniform (readfirstlane), so graph
// lookups stay scalar loads.  Small cache-resident chunks (generic_decode) use 64 threads x V = 1..4.
template <int V>
__device__ __forceinline__ bool tile_slot(int nodes, int tpl2, int64_t B, int& node, int64_t& cw) {
    node = __builtin_amdgcn_readfirstlane((int)(blockIdx.y << (8 - tpl2)) + (int)(threadIdx.x >> tpl2));
    cw = (((int64_t)blockIdx.x << tpl2) + (int64_t)(threadIdx.x & ((1u << tpl2) - 1u))) * V;
    return node < nodes && cw < B;
}

// Message streams are read once and written once per iteration: GEN_NT_LOAD / GEN_NT_STORE build
// variants with non-temporal ("nt") cache policy on them (A/B, scripts/mkvariant.sh).
#ifndef GEN_NT_LOAD
#define GEN_NT_LOAD 0
#endif
// GEN_SKIP_DUP: the min-sum kernels load only the d < MAXD edges a node has (d is wave-uniform: a scalar
// branch per slot) instead of re-loading the last edge into the unused slots (cache hits, but TA / L2 requests:
// DVB-S2's variables have degree 8, 3 or 2 under MAXD = 8)
#ifndef GEN_VW_CAP
#define GEN_VW_CAP 16  // A/B knob: at most this many codewords per thread in the streaming kernels' wide tiles
#endif
#ifndef GEN_TPL2_MAX
#define GEN_TPL2_MAX 8  // A/B knob: at most 2^GEN_TPL2_MAX threads per node (the rest of the 256 take other nodes)
#endif
#ifndef GEN_SKIP_DUP
#define GEN_SKIP_DUP 0
#endif
#ifndef GEN_NT_STORE
#define GEN_NT_STORE 0
#endif

template <typename T, int V>
struct Vec {
    T x[V];
};
template <typename T, int V>
__device__ __forceinline__ Vec<T, V> vload(const T* p) {
    Vec<T, V> r;
    if constexpr (V * sizeof(T) == 16) {
        using U = __attribute__((ext_vector_type(4))) float;
        const U u = GEN_NT_LOAD ? __builtin_nontemporal_load(reinterpret_cast<const U*>(p)) : *reinterpret_cast<const U*>(p);
        __builtin_memcpy(r.x, &u, 16);
    } else if constexpr (V * sizeof(T) == 8) {
        using U = __attribute__((ext_vector_type(2))) float;
        const U u = GEN_NT_LOAD ? __builtin_nontemporal_load(reinterpret_cast<const U*>(p)) : *reinterpret_cast<const U*>(p);
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
        if constexpr (GEN_NT_STORE) __builtin_nontemporal_store(u, reinterpret_cast<U*>(p));
        else *reinterpret_cast<U*>(p) = u;
    } else if constexpr (V * sizeof(T) == 8) {
        using U = __attribute__((ext_vector_type(2))) float;
        U u;
        __builtin_memcpy(&u, r.x, 8);
        if constexpr (GEN_NT_STORE) __builtin_nontemporal_store(u, reinterpret_cast<U*>(p));
        else *reinterpret_cast<U*>(p) = u;
    } else {
#pragma unroll
        for (int i = 0; i < V; ++i) p[i] = r.x[i];
    }
}

// Early stop: codewords whose syndrome was zero are frozen (their c2v is never written again).
template <int V>
__device__ __forceinline__ bool all_done(const uint8_t* done) {
    bool a = true;
#pragma unroll
    for (int i = 0; i < V; ++i) a = a && done[i];
    return a;
}
template <typename T, int V, bool ES>
__device__ __forceinline__ void store_live(T* p, const Vec<T, V>& r, const uint8_t* done) {
    if constexpr (!ES) {
        vstore<T, V>(p, r);
    } else {
        bool any = false;
#pragma unroll
        for (int i = 0; i < V; ++i) any = any || done[i];
        if (!any) {
            vstore<T, V>(p, r);
        } else {
#pragma unroll
            for (int i = 0; i < V; ++i)
                if (!done[i]) p[i] = r.x[i];
        }
    }
}

// Syndrome of the hard decisions hb[n][ldb] (written by the VN kernel from APP_it): one thread per
// (check, 4 codewords); any odd check marks its codeword unsatisfied (all writers store 1: benign).
template <int = 0>  // a template: defined in every including unit without duplicate symbols
__global__ __launch_bounds__(256) void k_syndrome(const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col_idx,
                                                  const uint8_t* __restrict__ hb, const uint8_t* __restrict__ done,
                                                  uint8_t* __restrict__ unsat, int64_t B, int64_t ldb) {
    const int c = blockIdx.y;
    const int64_t cw = ((int64_t)blockIdx.x * kTB + threadIdx.x) * 4;
    if (cw >= B) return;
    const uint32_t dn = *reinterpret_cast<const uint32_t*>(done + cw);
    if (dn == 0x01010101u) return;
    uint32_t par = 0;
    for (int e = row_ptr[c]; e < row_ptr[c + 1]; ++e)
        par ^= *reinterpret_cast<const uint32_t*>(hb + (int64_t)col_idx[e] * ldb + cw);
    par &= 0x01010101u;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if ((par >> (8 * i)) & 1u) unsat[cw + i] = 1;
}

// After the syndrome of APP_it (it >= 1): converged codewords become done with iters_used = it.
template <int = 0>  // a template: defined in every including unit without duplicate symbols
__global__ __launch_bounds__(256) void k_converge(uint8_t* __restrict__ done, uint8_t* __restrict__ unsat,
                                                  int32_t* __restrict__ used, int64_t B, int it) {
    const int64_t cw = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cw >= B) return;
    if (!done[cw] && !unsat[cw]) {
        done[cw] = 1;
        used[cw] = it;
    }
    unsat[cw] = 0;
}

template <int = 0>  // a template: defined in every including unit without duplicate symbols
__global__ __launch_bounds__(256) void k_used_final(const uint8_t* __restrict__ done, int32_t* __restrict__ used,
                                                    int64_t B, int iters) {
    const int64_t cw = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cw < B && !done[cw]) used[cw] = iters;
}

// Loads are issued for all MAXD slots with the edge index clamped to the last valid one (harmless
// duplicate reads): a wave-uniform `if (k < d)` around each load makes hipcc branch around it and
// drain vmcnt per load (cdna_hip_programming.md §5, load-reduce trap (c)).

template <typename T, int MAXD, bool ES, int V>
__global__ __launch_bounds__(256) void k_vn_sp(const int32_t* __restrict__ var_ptr, const int32_t* __restrict__ var_edges,
                                               const T* __restrict__ L, const T* __restrict__ c2v, T* __restrict__ v2c,
                                               int64_t B, int64_t ldb, int first, uint8_t* __restrict__ hb,
                                               const uint8_t* __restrict__ done, int nodes, int tpl2) {
    int v;
    int64_t cw;
    if (!tile_slot<V>(nodes, tpl2, B, v, cw)) return;
    if (ES && all_done<V>(done + cw)) return;
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
    if constexpr (std::is_same_v<T, float>) {
        // O(d) exclusive sums in log2 units, common.h vn_excl_sums's order (suffix right to left, prefix left to
        // right, S_t = P_t + Q_{t+1}) at this node's run-time degree d
        float Q[MAXD][V];
        static_for<1, MAXD>([&](auto ii) __attribute__((always_inline)) {
            constexpr int u = MAXD - decltype(ii)::value;  // MAXD-1 .. 1
#pragma unroll
            for (int i = 0; i < V; ++i) {
                if (u == d - 1) Q[u][i] = x[u].x[i];
                else if constexpr (u + 1 < MAXD) Q[u][i] = Q[u + 1][i] + x[u].x[i];  // used only when u < d - 1
            }
        });
        static_for<0, MAXD>([&](auto tt) __attribute__((always_inline)) {
            constexpr int t = decltype(tt)::value;
            if (t < d) {
                Vec<T, V> o;
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    float S;
                    if constexpr (t == 0) S = d == 1 ? 0.0f : Q[1][i];
                    else if constexpr (t + 1 < MAXD) S = t == d - 1 ? P.x[i] : P.x[i] + Q[t + 1][i];
                    else S = P.x[i];
                    o.x[i] = vn_signed_a(sp_vn_arg(Lv.x[i], S));
                    P.x[i] = t == 0 ? x[0].x[i] : P.x[i] + x[t].x[i];
                }
                vstore<T, V>(v2c + off[t], o);
            }
        });
        if constexpr (ES) {  // z of APP_it from the ascending sum 0 + x_0 + ... (the register kernels' zcol)
#pragma unroll
            for (int i = 0; i < V; ++i) {
                float Sa = 0.0f;
#pragma unroll
                for (int k = 0; k < MAXD; ++k)
                    if (k < d) Sa += x[k].x[i];
                hb[(int64_t)v * ldb + cw + i] = (uint8_t)Num<T>::bit(sp_z<T>(Lv.x[i], Sa));
            }
        }
        return;
    }
    // slots by static_for: x[] / off[] indices are constants (with #pragma unroll the V = 2 bodies were
    // left rolled and x[] went to scratch)
    static_for<0, MAXD>([&](auto tt) __attribute__((always_inline)) {
        constexpr int t = decltype(tt)::value;
        if (t < d) {
            Vec<T, V> o;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                T S = P.x[i];
                static_for<t + 1, MAXD>([&](auto uu) __attribute__((always_inline)) {
                    constexpr int u = decltype(uu)::value;
                    if (u < d) S += x[u].x[i];
                });
                o.x[i] = Num<T>::tanh_(T(0.5) * (Lv.x[i] + S));  // fp64: the reference's operations
                P.x[i] += x[t].x[i];
            }
            vstore<T, V>(v2c + off[t], o);
        }
    });
    if constexpr (ES) {  // hard decision of APP_it = the final layer's z (bp.py:36-39,51)
#pragma unroll
        for (int i = 0; i < V; ++i) hb[(int64_t)v * ldb + cw + i] = (uint8_t)Num<T>::bit(sp_z<T>(Lv.x[i], P.x[i]));
    }
}

// Weighted VC + tanh (bp_vc.py:16-27 with input_weight / llr_weight != 1): every target slot sums its own
// weighted sources skipping itself — fp64: ascending, the masked mm's terms in its k order; fp32: the sources
// before it left to right plus the sources after it right to left, the association of the unweighted O(d) sums
// (common.h vn_excl_sums), so unit weights give the unweighted messages bit for bit.  Weights are wave-uniform
// (scalar loads).  vn_it/lw_it point at this iteration's block (null = ones).
template <typename T, int MAXD, int V>
__global__ __launch_bounds__(256) void k_vn_spw(const int32_t* __restrict__ var_ptr, const int32_t* __restrict__ var_edges,
                                                const int32_t* __restrict__ wofs, const T* __restrict__ vn_it,
                                                const T* __restrict__ lw_it, const T* __restrict__ L,
                                                const T* __restrict__ c2v, T* __restrict__ v2c, int64_t B, int64_t ldb,
                                                int first, int nodes, int tpl2) {
    int v;
    int64_t cw;
    if (!tile_slot<V>(nodes, tpl2, B, v, cw)) return;
    const int a = var_ptr[v];
    const int d = var_ptr[v + 1] - a;
    if (d == 0) return;
    const T* wv = vn_it ? vn_it + wofs[v] : nullptr;
    const T lw = lw_it ? lw_it[v] : T(1);
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
#pragma unroll
    for (int t = 0; t < MAXD; ++t)
        if (t < d) {
            Vec<T, V> o;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                if constexpr (std::is_same_v<T, float>) {
                    float P = 0.0f, Q = 0.0f;
                    bool hp = false, hq = false;
#pragma unroll
                    for (int u = MAXD - 1; u >= 0; --u)
                        if (u < d && u > t) {
                            const float y = (wv ? wv[t * d + u] : 1.0f) * x[u].x[i];
                            Q = hq ? Q + y : y;
                            hq = true;
                        }
#pragma unroll
                    for (int u = 0; u < MAXD; ++u)
                        if (u < t) {
                            const float y = (wv ? wv[t * d + u] : 1.0f) * x[u].x[i];
                            P = hp ? P + y : y;
                            hp = true;
                        }
                    const float S = hp ? (hq ? P + Q : P) : (hq ? Q : 0.0f);
                    o.x[i] = vn_signed_a(sp_vn_arg(lw * Lv.x[i], S));
                } else {
                    T S = T(0);
#pragma unroll
                    for (int u = 0; u < MAXD; ++u)
                        if (u < d && u != t) S += (wv ? wv[t * d + u] : T(1)) * x[u].x[i];
                    o.x[i] = Num<T>::tanh_(T(0.5) * (lw * Lv.x[i] + S));
                }
            }
            vstore<T, V>(v2c + off[t], o);
        }
}

// zf[b] = 1 iff codeword b's LLRs hold an exact zero (+-0): the codewords the a == 1 rule applies to (common.h, the
// rule is per codeword).  One wave per codeword; the same test as the register kernels' k_sp_zero_scan.
template <int = 0>
__global__ __launch_bounds__(256) void k_zero_flags(const float* __restrict__ llr, int64_t B, int n,
                                                    uint8_t* __restrict__ zf) {
    const int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (b >= B) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const float* p = llr + b * n;
    bool z = false;
    for (int i = lane; i < n; i += 64) z |= p[i] == 0.0f;
    const bool any = __ballot(z) != 0;
    if (lane == 0) zf[b] = any ? 1 : 0;
}

template <typename T, int MAXD, bool ES, int V>
__global__ __launch_bounds__(256) void k_cn_sp(const int32_t* __restrict__ row_ptr, const T* __restrict__ v2c,
                                               T* __restrict__ c2v, int64_t B, int64_t ldb, T clamp,
                                               const uint8_t* __restrict__ done, int nodes, int tpl2,
                                               const uint8_t* __restrict__ zf) {
    int c;
    int64_t cw;
    if (!tile_slot<V>(nodes, tpl2, B, c, cw)) return;
    if (ES && all_done<V>(done + cw)) return;
    const int a = row_ptr[c];
    const int d = row_ptr[c + 1] - a;
    if (d == 0) return;  // an empty check carries no messages
    Vec<T, V> t[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) t[k] = vload<T, V>(v2c + (int64_t)(a + (k < d ? k : d - 1)) * ldb + cw);
    if constexpr (std::is_same_v<T, float>) {
        // (D, S) form: slots >= d carry a = 0, whose set is the identity, so every slot runs the same code
        const float cmax2 = sp_cmax2(clamp);  // messages in log2 units (common.h)
        DSet suf[MAXD + 1][V];
        uint32_t sg[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
            suf[MAXD][i] = ds_identity();
            sg[i] = 0;
        }
        static_for<0, MAXD>([&](auto kk) __attribute__((always_inline)) {
            constexpr int u = MAXD - 1 - decltype(kk)::value;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                suf[u][i] = ds_push(suf[u + 1][i], u < d ? fabsf(t[u].x[i]) : 0.0f);
                sg[i] ^= u < d ? f2u(t[u].x[i]) : 0u;
            }
        });
        DSet pre[V];
        int n1[V];  // edges with a == 1: every other edge outputs exactly +-0 (common.h ds_fix_one), in the codewords
                    // whose LLRs hold an exact zero (zf: the rule is per codeword); none counted elsewhere
#pragma unroll
        for (int i = 0; i < V; ++i) {
            pre[i] = ds_identity();
            n1[i] = 0;
            const bool fx = zf[cw + i] != 0;
#pragma unroll
            for (int k = 0; k < MAXD; ++k) n1[i] += (fx && k < d && fabsf(t[k].x[i]) == 1.0f) ? 1 : 0;
        }
        static_for<0, MAXD>([&](auto ee) __attribute__((always_inline)) {
            constexpr int e = decltype(ee)::value;
            if (e < d) {
                Vec<T, V> o;
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    o.x[i] = ds_join_out(pre[i], suf[e + 1][i], sg[i] ^ f2u(t[e].x[i]), cmax2);
                    if (n1[i] - (fabsf(t[e].x[i]) == 1.0f ? 1 : 0) > 0) o.x[i] = u2f(f2u(o.x[i]) & 0x80000000u);
                    pre[i] = ds_push(pre[i], fabsf(t[e].x[i]));
                }
                store_live<T, V, ES>(c2v + (int64_t)(a + e) * ldb + cw, o, done + cw);
            }
        });
        return;
    }
    Vec<T, V> Q;
#pragma unroll
    for (int i = 0; i < V; ++i) Q.x[i] = T(1);
    static_for<0, MAXD>([&](auto ee) __attribute__((always_inline)) {  // constant slot indices (see k_vn_sp)
        constexpr int e = decltype(ee)::value;
        if (e < d) {
            Vec<T, V> o;
#pragma unroll
            for (int i = 0; i < V; ++i) {
                T p = Q.x[i];
                static_for<e + 1, MAXD>([&](auto uu) __attribute__((always_inline)) {
                    constexpr int u = decltype(uu)::value;
                    if (u < d) p *= t[u].x[i];
                });
                o.x[i] = cn_tanh_out(p, clamp);  // clamp p, log((1+p)/(1-p)), clamp (common.h)
                Q.x[i] *= t[e].x[i];
            }
            store_live<T, V, ES>(c2v + (int64_t)(a + e) * ldb + cw, o, done + cw);
        }
    });
}

template <int MAXD, bool ES, int V>
__global__ __launch_bounds__(256) void k_vn_ms(const int32_t* __restrict__ var_ptr, const int32_t* __restrict__ var_edges,
                                               const float* __restrict__ L, const float* __restrict__ c2v,
                                               float* __restrict__ v2c, int64_t B, int64_t ldb, int first,
                                               uint8_t* __restrict__ hb, const uint8_t* __restrict__ done, int nodes,
                                               int tpl2) {
    int v;
    int64_t cw;
    if (!tile_slot<V>(nodes, tpl2, B, v, cw)) return;
    if (ES && all_done<V>(done + cw)) return;
    const int a = var_ptr[v];
    const int d = var_ptr[v + 1] - a;
    if (d == 0) return;
    Vec<float, V> app = vload<float, V>(L + (int64_t)v * ldb + cw);
    Vec<float, V> x[MAXD];
    int64_t off[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        off[k] = (int64_t)var_edges[a + (k < d ? k : d - 1)] * ldb + cw;
        if (GEN_SKIP_DUP && k >= d) continue;  // d is wave-uniform: a scalar branch, the loop stays unrolled
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
    if constexpr (ES) {
#pragma unroll
        for (int i = 0; i < V; ++i) hb[(int64_t)v * ldb + cw + i] = (uint8_t)(0.5f * app.x[i] <= kZthrF32);
    }
}

template <int MAXD, bool ES, int V>
__global__ __launch_bounds__(256) void k_cn_ms(const int32_t* __restrict__ row_ptr, const float* __restrict__ v2c,
                                               float* __restrict__ c2v, int64_t B, int64_t ldb, float clamp,
                                               float alpha, float beta, const uint8_t* __restrict__ done, int nodes,
                                               int tpl2) {
    int c;
    int64_t cw;
    if (!tile_slot<V>(nodes, tpl2, B, c, cw)) return;
    if (ES && all_done<V>(done + cw)) return;
    const int a = row_ptr[c];
    const int d = row_ptr[c + 1] - a;
    if (d == 0) return;
    Vec<float, V> t[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (GEN_SKIP_DUP && k >= d) continue;  // d is wave-uniform: a scalar branch, the loop stays unrolled
        t[k] = vload<float, V>(v2c + (int64_t)(a + (k < d ? k : d - 1)) * ldb + cw);
    }
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
        if (k < d) store_live<float, V, ES>(c2v + (int64_t)(a + k) * ldb + cw, t[k], done + cw);
}

// Final VC + sigmoid + hard decision (bp/bp.py:36-39,51; ofdm_functions.py:161), transposed back to
// the caller's [B][n] layout through an LDS tile.
template <typename T, int MAXD, bool MS>
__global__ __launch_bounds__(256) void k_final(const int32_t* __restrict__ var_ptr, const int32_t* __restrict__ var_edges,
                                               const T* __restrict__ L, const T* __restrict__ c2v, int64_t B,
                                               int64_t ldb, int n, uint8_t* __restrict__ bits, T* __restrict__ soft,
                                               int soft_z, const T* __restrict__ fin, const T* __restrict__ flw) {
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
                for (int k = 0; k < d; ++k)
                    S += (fin ? fin[a + k] : T(1)) * c2v[(int64_t)var_edges[a + k] * ldb + cw];
                z = sp_z<T>((flw ? flw[v] : T(1)) * Lv, S);  // fp32: S in log2 units
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

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace: L[n][ldb], v2c[E][ldb], c2v[E][ldb] (elem bytes each) and, with early stop,
// hb[n][ldb] (uint8 hard decisions), done[ldb], unsat[ldb], used[ldb] (int32 scratch).
struct WsLayout {
    size_t L, v2c, c2v, hb, done, unsat, used, zf, total;
};
static WsLayout layout(const GenericArgs& g, int64_t B, size_t elem, bool es) {
    const int64_t ldb = (B + 63) / 64 * 64;
    WsLayout w{};
    size_t off = 0;
    w.L = off;
    off += a256(elem * (size_t)ldb * g.n);
    w.v2c = off;
    off += a256(elem * (size_t)ldb * g.E);
    w.c2v = off;
    off += a256(elem * (size_t)ldb * g.E);
    if (es) {
        w.hb = off;
        off += a256((size_t)ldb * g.n);
        w.done = off;
        off += a256((size_t)ldb);
        w.unsat = off;
        off += a256((size_t)ldb);
        w.used = off;
        off += a256((size_t)ldb * 4);
    }
    w.zf = off;  // fp32 tanh-SP: one byte per codeword, an exact-zero LLR (the a == 1 rule's codewords, k_zero_flags)
    off += a256((size_t)ldb);
    w.total = off;
    return w;
}

// Cache-resident chunks.  A decode of B codewords may run as consecutive chunks of Bc codewords whose
// per-iteration working set (L, v2c, c2v: elem * (n + 2E) bytes per codeword) fits the 256 MiB Infinity
// Cache, so from the second iteration on the message streams are served on-die.  Chunks are independent
// (codewords never interact), so results do not depend on Bc (tests/test_gpu_parity.py).
// Measured (profiles/r01/cache_sweep.txt): min-sum (648,1/2) generic 2.45M -> 2.99M cw/s at 192 MB
// (VN 4.5 -> 6.9 TB/s, CN 5.9 -> 7.3 TB/s effective); no gain where a chunk would need narrow tiles
// (DVB-S2-size codes: Bc = 64) and a loss for tanh-SP (more launches, no bandwidth to win).  Default:
// min-sum only, 192 MB, only when chunks keep full wide tiles (Bc >= 1024).  LDPC_CACHE_BUDGET_MB
// overrides for every algorithm (0 = one pass).
static int64_t chunk_cw(const GenericArgs& g, int64_t B, const ldpc_params& p) {
    const size_t elem = (p.flags & LDPC_F_F64) ? 8 : 4;
    const bool es = (p.flags & LDPC_F_EARLY_STOP) != 0;
    const char* env = getenv("LDPC_CACHE_BUDGET_MB");  // read per call: tests and benches vary it
    int64_t budget, min_bc;
    if (env) {
        const long v = atol(env);
        budget = (int64_t)(v < 0 ? 0 : v) << 20;
        min_bc = 64;
    } else {
        budget = (p.algo == LDPC_ALGO_MIN_SUM) ? (int64_t)192 << 20 : 0;
        min_bc = 1024;
    }
    if (budget == 0) return B;
    const int64_t per_cw = (int64_t)elem * (g.n + 2 * (int64_t)g.E) + (es ? g.n : 0);
    const int64_t bc = budget / per_cw / 64 * 64;
    if (bc < min_bc) return env ? min_bc : B;
    return bc < B ? bc : B;
}


// One driver for both algorithms: VN and CN kernels per iteration (plus, with early stop, the
// syndrome of APP_it and the convergence update between them), then the final decision kernel.
template <typename T, bool MS, bool ES>
static int run(const GenericArgs& g, const T* llr_dev, int64_t B, const ldpc_params& p, uint8_t* bits, T* soft,
               int32_t* iters_used, char* ws, hipStream_t st, const BPWeights* wts) {
    const int64_t ldb = (B + 63) / 64 * 64;
    const WsLayout w = layout(g, B, sizeof(T), ES);
    T* L = (T*)(ws + w.L);
    T* v2c = (T*)(ws + w.v2c);
    T* c2v = (T*)(ws + w.c2v);
    uint8_t* hb = ES ? (uint8_t*)(ws + w.hb) : nullptr;
    uint8_t* done = ES ? (uint8_t*)(ws + w.done) : nullptr;
    uint8_t* unsat = ES ? (uint8_t*)(ws + w.unsat) : nullptr;
    int32_t* used = ES ? (iters_used ? iters_used : (int32_t*)(ws + w.used)) : nullptr;
    const int soft_z = (p.flags & LDPC_F_SOFT_Z) ? 1 : 0;
    const T clamp = (T)p.clamp;
    const dim3 tb(kTB);
    const unsigned gcw = (unsigned)((B + kTB - 1) / kTB);
    const T unit = (!MS && std::is_same_v<T, float>) ? T(kLog2eF32) : T(1);  // fp32 tanh-SP messages: log2 units
    k_load_llr<T><<<dim3((unsigned)((B + 63) / 64), (g.n + 63) / 64), tb, 0, st>>>(llr_dev, L, B, g.n, ldb, T(-1));
    uint8_t* zf = (uint8_t*)(ws + w.zf);
    if constexpr (!MS && std::is_same_v<T, float>)
        k_zero_flags<><<<(unsigned)((B + 3) / 4), tb, 0, st>>>((const float*)llr_dev, B, g.n, zf);
    // non-zero initial messages x (bp/bp.py:43-47): iteration 0 reads them like any later iteration
    const T* x0 = wts ? (const T*)wts->c2v0 : nullptr;
    if (x0) k_load_llr<T><<<dim3((unsigned)((B + 63) / 64), (g.E + 63) / 64), tb, 0, st>>>(x0, c2v, B, g.E, ldb, unit);
    if (ES) {
        if (hipMemsetAsync(done, 0, (size_t)ldb, st) != hipSuccess || hipMemsetAsync(unsat, 0, (size_t)ldb, st) != hipSuccess)
            return set_error(LDPC_EHIP, "early-stop state init failed");
    }
    const int dv = pick_maxd(g.max_dv), dc = pick_maxd(g.max_dc);
    if (dv < 0 || dc < 0) return set_error(LDPC_EUNSUPPORTED, "node degree > 32 not supported by generic kernels");
    const T* w_vn = wts ? (const T*)wts->vn : nullptr;
    const T* w_lw = wts ? (const T*)wts->lw : nullptr;
    // tiles: wide (V = VW codewords per thread) when a wave's 64 lanes have >= 64*VW codewords to cover,
    // else narrow (V = 1); 2^tpl2 threads per node
    auto tile = [B](int vw, int& V, int& tpl2) {
        vw = vw < GEN_VW_CAP ? vw : GEN_VW_CAP;
        V = (B >= 64 * vw) ? vw : 1;
        const int64_t lanes = (B + V - 1) / V;
        tpl2 = lanes > 128 ? 8 : lanes > 64 ? 7 : 6;
        tpl2 = tpl2 < GEN_TPL2_MAX ? tpl2 : GEN_TPL2_MAX;
    };
    auto grid = [B](int V, int tpl2, int nodes) {
        return dim3((unsigned)((B + ((int64_t)V << tpl2) - 1) / ((int64_t)V << tpl2)),
                    (unsigned)((nodes + (256 >> tpl2) - 1) / (256 >> tpl2)));
    };
    for (int it = 0; it < p.iters; ++it) {
        const int first = (it == 0) && !x0;
        if (!MS && wts && (wts->vn || wts->lw)) {
            const T* vn_it = w_vn ? w_vn + (int64_t)it * g.W : nullptr;
            const T* lw_it = w_lw ? w_lw + (int64_t)it * g.n : nullptr;
#define VNW1(D, VV) \
    k_vn_spw<T, D, VV><<<grid(VV, tpl2, g.n), tb, 0, st>>>(g.var_ptr, g.var_edges, g.wofs, vn_it, lw_it, L, c2v, v2c, B, ldb, first, g.n, tpl2)
#define VNW(D)                                                     \
    do {                                                           \
        int V, tpl2;                                               \
        tile(VW<T, D>::value, V, tpl2);                            \
        if (V == 1) VNW1(D, 1); else VNW1(D, (VW<T, D>::value));   \
    } while (0)
            switch (dv) { case 4: VNW(4); break; case 8: VNW(8); break; case 12: VNW(12); break; case 16: VNW(16); break; case 20: VNW(20); break; case 24: VNW(24); break; default: VNW(32); }
#undef VNW
#undef VNW1
        } else {
#define VN1(D, VV)                                                                                                  \
    do {                                                                                                           \
        if constexpr (MS)                                                                                          \
            k_vn_ms<D, ES, VV><<<grid(VV, tpl2, g.n), tb, 0, st>>>(g.var_ptr, g.var_edges, (const float*)L,          \
                (const float*)c2v, (float*)v2c, B, ldb, first, hb, done, g.n, tpl2);                              \
        else                                                                                                       \
            k_vn_sp<T, D, ES, VV><<<grid(VV, tpl2, g.n), tb, 0, st>>>(g.var_ptr, g.var_edges, L, c2v, v2c,          \
                B, ldb, first, hb, done, g.n, tpl2);                                                               \
    } while (0)
#define VN(D)                                                      \
    do {                                                           \
        int V, tpl2;                                               \
        tile(VW<T, D>::value, V, tpl2);                            \
        if (V == 1) VN1(D, 1); else VN1(D, (VW<T, D>::value));     \
    } while (0)
        switch (dv) { case 4: VN(4); break; case 8: VN(8); break; case 12: VN(12); break; case 16: VN(16); break; case 20: VN(20); break; case 24: VN(24); break; default: VN(32); }
#undef VN
#undef VN1
        }
        if (ES && it > 0) {  // the oracle tests the syndrome of APP after each iteration >= 1
            k_syndrome<><<<dim3((unsigned)((B + 4 * kTB - 1) / (4 * kTB)), g.m), tb, 0, st>>>(g.row_ptr, g.col_idx, hb,
                                                                                          done, unsat, B, ldb);
            k_converge<><<<gcw, tb, 0, st>>>(done, unsat, used, B, it);
        }
#define CN1(D, VV)                                                                                                  \
    do {                                                                                                           \
        if constexpr (MS)                                                                                          \
            k_cn_ms<D, ES, VV><<<grid(VV, tpl2, g.m), tb, 0, st>>>(g.row_ptr, (const float*)v2c, (float*)c2v, B, ldb, \
                p.clamp, p.alpha, p.beta, done, g.m, tpl2);                                                        \
        else                                                                                                       \
            k_cn_sp<T, D, ES, VV><<<grid(VV, tpl2, g.m), tb, 0, st>>>(g.row_ptr, v2c, c2v, B, ldb, clamp, done, g.m, tpl2, zf); \
    } while (0)
#define CN(D)                                                      \
    do {                                                           \
        int V, tpl2;                                               \
        tile(VW<T, D>::value, V, tpl2);                            \
        if (V == 1) CN1(D, 1); else CN1(D, (VW<T, D>::value));     \
    } while (0)
        switch (dc) { case 4: CN(4); break; case 8: CN(8); break; case 12: CN(12); break; case 16: CN(16); break; case 20: CN(20); break; case 24: CN(24); break; default: CN(32); }
#undef CN
#undef CN1
    }
    if (p.iters == 0 && !x0) (void)hipMemsetAsync(c2v, 0, sizeof(T) * (size_t)g.E * ldb, st);
    k_final<T, 32, MS><<<dim3((unsigned)((B + 63) / 64), (g.n + 63) / 64), tb, 0, st>>>(g.var_ptr, g.var_edges, L, c2v, B,
                                                                                      ldb, g.n, bits, soft, soft_z,
                                                                                      wts ? (const T*)wts->fin : nullptr,
                                                                                      wts ? (const T*)wts->flw : nullptr);
    if (ES) {
        k_used_final<><<<gcw, tb, 0, st>>>(done, used, B, p.iters);
    } else if (iters_used) {
        fill_i32(iters_used, B, p.iters, st);  // every codeword runs the fixed iteration count
    }
    return LDPC_OK;
}

}  // namespace ldpc
