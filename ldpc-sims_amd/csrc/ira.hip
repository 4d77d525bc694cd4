// ira.hip — min-sum decoder for IRA codes with the DVB-S2 structure (EN 302 307 §5.3.2: information bit m of
// group g is accumulated into parity addresses (x + m q) mod M for every x of the group's table row; parity
// staircase p_j ^= p_{j-1}), BASELINE config [4]: DVB-S2 64800 rate 1/2, 50 min-sum iterations.
//
// Why a kernel of its own.  The generic CSR kernels (generic_impl.h) stream every message through HBM each
// iteration — 16E + 4n bytes per codeword-iteration, 3.89 MB for DVB-S2 — and run at 0.85 of the chip's
// streaming rate: the byte count is the bound.  Relabelling check j = a + q b as (row a, position b) turns the
// code into a quasi-cyclic one with Z = 360: information edge (g, t) with table address x_t connects variable
// (g, m) to check (a_t, (s_t + m) mod 360), a_t = x_t mod q, s_t = x_t div q; the staircase connects parity
// (a, b) to checks (a, b) and its successor.  Lanes run over the 360 positions of one row of ONE codeword, so
// every access is a contiguous row segment (with one wrap) of a codeword-local array, whatever the batch.
//
// Dataflow (flooding, the oracle's operation order — oracle/numpy_ref.py ms, oracle/ldpc_oracle.c ms_f32):
//   check state  per check: mag1, mag2 (the two output magnitudes after ms_mag), meta = argmin slot (bits
//                27..31) | sign bit of every slot's c2v (bit s) — the exact c2v of every edge in 12 bytes
//   k_ira_vn     app_v = L_v + sum of v's c2v in ASCENDING CHECK order (decompressed from the check states)
//   k_ira_cn     v2c = app_v - c2v_old (decompressed from its own state), two-minimum, new state
// which are the oracle's VN (app = L + sum x_k; v2c = app - x_k) and CN bit for bit: the CN's order statistics
// and sign XOR do not depend on the slot order (an argmin tie has min2 == min1, so either slot gets the same
// magnitude), and the VN sums in the oracle's order — for an information variable the ascending check order
// of its d edges is the x-sorted table row rotated by the number of edges whose position wraps (b = s_t + m
// >= 360 gives the smaller check index), a per-lane barrel rotation.
// Bytes per codeword-iteration beyond L2 (each codeword's tasks run on one XCD back to back, so the
// re-reads of its check states and posteriors hit L2): L (4n) + states (12M) + app (4n) in the VN, app (4n)
// + states read and written (24M) in the CN = 16n + 36M = 2.1 MB for DVB-S2 1/2, against 3.89 MB for the
// two-array dataflow.  A chunk of codewords whose arrays (8n + 16M bytes each) fit the Infinity Cache decodes
// all its iterations before the next chunk starts; chunks go round-robin over two streams.  Also here: the parity
// posteriors formed by the check kernel (IRA_CNPAR) and early termination (IraEs) — DESIGN.md §3.8.
#include <stdlib.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "common.h"

namespace ldpc {

constexpr int kIZ = 360;       // DVB-S2 lifting (normal and short frames)
constexpr int kIVS = 16;       // table stride: information-variable degree bound
constexpr int kICS = 24;       // table stride: information slots per check bound
constexpr int kIPS = 24;       // parity slots: kIPS (p_j) and kIPS + 1 (p_{j-1}); meta bits 0..25, argmin 27..31

struct IRASpec {
    int q = 0, G = 0, k = 0, n = 0, M = 0, E = 0, maxdv = 0, maxr = 0, device = 0;
    int32_t *vn = nullptr, *vdeg = nullptr, *cn = nullptr, *cdeg = nullptr;  // device tables
};

// The tables are read-only for the whole decode: read through the constant address space so that every (uniform)
// table read is a scalar load.  As plain global pointers the compiler could not rule out that the kernels' own stores
// (app, states) alias them and read several rows with vector loads plus a wait and readfirstlane — one extra
// dependent round trip per task (round 6).
using cint32 = const __attribute__((address_space(4))) int32_t;
struct IRADev {
    cint32 *vn, *vdeg, *cn, *cdeg;
    int q, G, k, n, M;
};

// One check's state, 12 bytes read and written as one dwordx3: the two output magnitudes and the meta word
struct IraState {
    float m1, m2;
    uint32_t meta;
};
static_assert(sizeof(IraState) == 12, "one dwordx3 per check state");

#if IRA_DIAG_S8
// the states as an array of 8-byte pairs indexed like the 12-byte array (the first two thirds of the buffer)
__device__ __forceinline__ IraState ira_ld_i(const IraState* __restrict__ base, int64_t i) {
    const float2 m = reinterpret_cast<const float2*>(base)[i];
    return IraState{m.x, m.y, __float_as_uint(m.x) & 0x3ffu};
}
__device__ __forceinline__ void ira_st_i(IraState* __restrict__ base, int64_t i, const IraState& s) {
    reinterpret_cast<float2*>(base)[i] = make_float2(s.m1, s.m2 + __uint_as_float(s.meta & 1u));
}
#else
__device__ __forceinline__ IraState ira_ld_i(const IraState* __restrict__ base, int64_t i) { return base[i]; }
__device__ __forceinline__ void ira_st_i(IraState* __restrict__ base, int64_t i, const IraState& s) { base[i] = s; }
#endif
__device__ __forceinline__ IraState ira_ld(const IraState* __restrict__ p) { return *p; }

// c2v of slot `slot` from a check state: the argmin slot gets mag2, every other mag1; sign bit from meta
__device__ __forceinline__ float ira_c2v(const IraState& st, int slot) {
    const float mag = ((st.meta >> 27) == (uint32_t)slot) ? st.m2 : st.m1;
    return u2f(f2u(mag) | ((st.meta << (31 - slot)) & 0x80000000u));
}

// Workgroup b -> (codeword, task): blocks b and b + 8 share an XCD (MI355X_MICROARCH.md §Workgroup dispatch),
// so the T tasks of a codeword get consecutive blocks of one XCD and its arrays stay in that XCD's L2 while
// its tasks run.  A speed choice only: any placement gives the same results.
__device__ __forceinline__ bool ira_task(int T, int Bc, int& cw, int& task) {
    const int b = blockIdx.x;
    const int kk = b >> 3;
    const int c = kk / T;
    cw = c * 8 + (b & 7);
    task = kk - c * T;
    return cw < Bc;
}

// IRA_VN_ROT (A/B knob, off): the ascending-order sum by a barrel rotation of the d c2v values (log2 d select stages —
// which the compiler turns into a compare chain per output, ~150 v_cmp / v_cndmask pairs with s_nop hazard waits
// per degree-8 task) instead of two masked passes (ira_vn_info)
#ifndef IRA_VN_ROT
#define IRA_VN_ROT 0
#endif
#ifndef IRA_VN_SCHED
#define IRA_VN_SCHED 1
#endif
#ifndef IRA_CN_SCHED
#define IRA_CN_SCHED 1
#endif
// c'[i] = c[(i + rho) mod D], rho < D, by log2(D) stages of selects (rotations compose additively mod D)
template <int D>
__device__ __forceinline__ void rotate_left(float (&c)[D], int rho) {
    static_for<0, 5>([&](auto BB) __attribute__((always_inline)) {
        constexpr int sh = 1 << decltype(BB)::value;
        if constexpr (sh < D) {
            const bool on = (rho & sh) != 0;
            float t[D];
#pragma unroll
            for (int i = 0; i < D; ++i) t[i] = on ? c[(i + sh) % D] : c[i];
#pragma unroll
            for (int i = 0; i < D; ++i) c[i] = t[i];
        }
    });
}

// Workgroup shape: one task at a time over kIraLanes threads (6 waves over the 360 positions; lanes past 360
// repeat the last position and store nothing), `tpw` tasks one after the other.  Every load of a task is issued
// before the first is used: a task waits on one memory round trip, not one per edge (A/B
// profiles/r05/ab/ab_c4_ira_restructure.txt).  Two tasks side by side per workgroup measured no faster
// (ab_c4_ira_tpp.txt), nor did several positions per lane (ab_c4_ira_ppl.txt).
constexpr int kIraLanes = 384;
#ifndef IRA_DIAG_NOPAR
#define IRA_DIAG_NOPAR 0  // DIAGNOSTIC BUILD ONLY (wrong results): the VN skips its parity tasks, to price them
#endif
// IRA_CNPAR: the check kernel forms the posterior of parity p(r, b) itself as soon as it has the new states of rows
// r and r + 1 (consecutive rows of one workgroup: the row loop carries row r's new state to row r + 1), with the
// variable kernel's operations, (L + c2v_r) + c2v_{r+1}; the variable kernel keeps only the parity rows that end a
// check workgroup's group (their r + 1 lives in another workgroup) — 15 of 90 for DVB-S2 1/2 at 6 rows per group.
// The posteriors it writes are the NEXT iteration's, while other check workgroups still read this iteration's: the
// parity posteriors ping-pong between two buffers (ParBuf), M floats per codeword more.  Bitwise the same.
#ifndef IRA_DIAG_VN4
#define IRA_DIAG_VN4 0  // DIAGNOSTIC BUILD ONLY (wrong results): information c2v read as 4 contiguous bytes, to price 12 -> 4
#endif
#ifndef IRA_CNPAR
#define IRA_CNPAR 1
#endif
#ifndef IRA_VN_PAIR
#define IRA_VN_PAIR 0  // variable kernel: two information tasks of one degree with their loads in flight together (A/B knob)
#endif
#ifndef IRA_CN_EXACT
// check kernel instances for at most 5 and 6 information slots: no gathers of padded slots (DVB-S2 1/2 has 5 per check;
// the MAXR = 8 instance loads 8).  Config [4] 59.0 -> 60.3k cw/s (profiles/r06/ab/ab_c4_ira_r6x.txt)
#define IRA_CN_EXACT 1
#endif
#ifndef IRA_CN_PF
#define IRA_CN_PF 0  // check kernel: row ra + 1's loads issued before row ra's arithmetic (A/B knob)
#endif
#ifndef IRA_DIAG_S8
#define IRA_DIAG_S8 0  // DIAGNOSTIC BUILD ONLY (wrong results): check states of 8 bytes (m1, m2; meta from m1's bits), to price 12 -> 8
#endif

// parity posteriors of codeword c, parity index j = r 360 + b: p[c stride + j]
struct ParBuf {
    float* p;
    int64_t stride;
};

// Early termination (LDPC_F_EARLY_STOP; the oracle's ms_f32: after iteration it the decisions of app_{it+1} are
// tested, and a codeword whose syndrome is zero stops with iters_used = it + 1).  CN(it), it >= 1, tests app_it —
// the posteriors it reads anyway — and each check workgroup stores "one of my checks fails" to its own word
// flg[cw][group] (CN(0), which tests nothing, stores 1); VN(it + 1) ORs the codeword's words: zero means converged
// at it (conv[cw] = it, nothing more runs for that codeword; its app_it stays in place — the parity part in the
// buffer of iteration it).  Plain stores to distinct words: one atomic per wave on a per-codeword word cost 27 %
// of the decode at low Eb/N0 (memory-side atomics on a contended address).
struct IraEs {
    int32_t* conv;  // per codeword of the chunk: 0 = running, else iterations used
    int32_t* flg;   // [codeword][check group]: some check of the group fails on the tested posteriors
    int ng;         // check groups per codeword
    int it;         // the iteration of this launch
};

// app of information variable (g, pos) of degree D: L + its c2v in ascending check order.  The table row is sorted by
// x = a + q s, i.e. by s, so the entries whose position wraps (b = s + pos >= 360: the smaller check indices) are a
// suffix of it, and the ascending order is: the wrapped entries in table order, then the others in table order —
// summed as two masked passes (x + (-0) == x bit for bit, so a skipped entry changes nothing), 4 VALU per entry.
// The state of check (ra, b) is addressed by a 32-bit byte offset from the codeword's first state (a scalar base).
template <int D>
struct VnIn {
    IraState st[D];
    bool w[D];
    float a;
};
// the loads of one information task (its D check states and L), all issued before any use
template <int D>
__device__ __forceinline__ void ira_vn_load(cint32* row, int64_t vo, int64_t so, int pos, const float* __restrict__ L,
                                            const IraState* __restrict__ S, VnIn<D>& in) {
    const int p = min(pos, kIZ - 1);
    const char* const Sb = reinterpret_cast<const char*>(S + so);
    static_for<0, D>([&](auto TT) __attribute__((always_inline)) {
        constexpr int t = decltype(TT)::value;
        const int e = row[t];  // wave-uniform: a scalar load
        const int ra = e & 0xff, sh = (e >> 8) & 0x1ff;
        int b = p + sh;
        in.w[t] = b >= kIZ;
        b -= in.w[t] ? kIZ : 0;
#if IRA_DIAG_S8
        (void)Sb;
        in.st[t] = ira_ld_i(S, so + ra * kIZ + b);
#else
        const uint32_t off = (uint32_t)(ra * kIZ + b) * (uint32_t)sizeof(IraState);
        in.st[t] = ira_ld(reinterpret_cast<const IraState*>(Sb + off));
#endif
    });
    in.a = L[vo + p];
}
// app = L + the c2v in ascending check order, stored
template <int D>
__device__ __forceinline__ void ira_vn_sum(cint32* row, int64_t vo, int pos, float* __restrict__ app, const VnIn<D>& in) {
    float c[D];
    static_for<0, D>([&](auto TT) __attribute__((always_inline)) {
        constexpr int t = decltype(TT)::value;
        c[t] = ira_c2v(in.st[t], row[t] >> 17);
    });
    float sum = in.a;
#if IRA_VN_ROT
    int wrapped = 0;
#pragma unroll
    for (int t = 0; t < D; ++t) wrapped += in.w[t];
    const int rho = wrapped == 0 ? 0 : D - wrapped;
    rotate_left<D>(c, rho);
#pragma unroll
    for (int t = 0; t < D; ++t) sum = sum + c[t];
#else
#pragma unroll
    for (int t = 0; t < D; ++t) sum = sum + (in.w[t] ? c[t] : -0.0f);
#pragma unroll
    for (int t = 0; t < D; ++t) sum = sum + (in.w[t] ? -0.0f : c[t]);
#endif
    if (pos < kIZ) app[vo + pos] = sum;
}
template <int D>
__device__ __forceinline__ void ira_vn_info(cint32* row, int64_t vo, int64_t so, int pos,
                                            const float* __restrict__ L, const IraState* __restrict__ S,
                                            float* __restrict__ app) {
#if IRA_DIAG_VN4
    const int p = min(pos, kIZ - 1);
    float c[D];
    bool w[D];
    const float a = L[vo + p];
    static_for<0, D>([&](auto TT) __attribute__((always_inline)) {
        constexpr int t = decltype(TT)::value;
        const int e = row[t];
        const int ra = e & 0xff, sh = (e >> 8) & 0x1ff, slot = e >> 17;
        int b = p + sh;
        w[t] = b >= kIZ;
        b -= w[t] ? kIZ : 0;
        const float x = reinterpret_cast<const float*>(S)[so + (int64_t)ra * kIZ + b];
        c[t] = ira_c2v(IraState{x, x, (uint32_t)slot << 27}, slot);
    });
    float sum = a;
#pragma unroll
    for (int t = 0; t < D; ++t) sum = sum + (w[t] ? c[t] : -0.0f);
#pragma unroll
    for (int t = 0; t < D; ++t) sum = sum + (w[t] ? -0.0f : c[t]);
    if (pos < kIZ) app[vo + pos] = sum;
#else
    VnIn<D> in;
    ira_vn_load<D>(row, vo, so, pos, L, S, in);
    // IRA_VN_SCHED: every state load issued before the first is consumed (the scheduler had interleaved the first
    // loads' decompression with the later loads' issue, behind a wait for the first ones: two round trips per task)
#if IRA_VN_SCHED
    __builtin_amdgcn_sched_barrier(0);
#endif
    ira_vn_sum<D>(row, vo, pos, app, in);
#endif
}

// One task = one variable group (information group g < G, or parity row a = g - G) of one codeword; lanes =
// the 360 positions.  Writes app in the permuted layout (information: g*360 + m, parity: k + a*360 + b).
// Parity rows: every row (pgrp = 0), or only the last row of each group of pgrp check rows (IRA_CNPAR: the check
// kernel formed the others); their posteriors go to `par`.
template <int MAXDV, bool ES>
__global__ __launch_bounds__(kIraLanes) void k_ira_vn(IRADev t, const float* __restrict__ L, float* __restrict__ app,
                                                      const IraState* __restrict__ S, ParBuf par, int pgrp,
                                                      int Bc, int tpw, IraEs es) {
    const int T = t.G + (pgrp > 0 ? (t.q + pgrp - 1) / pgrp : t.q);
    int cw, tb;
    if (!ira_task((T + tpw - 1) / tpw, Bc, cw, tb)) return;
    const int pos = threadIdx.x;
    if constexpr (ES) {  // (wave-uniform loads)
        if (es.conv[cw] != 0) return;
        if (es.it >= 1) {
            const int32_t* f = es.flg + (int64_t)cw * es.ng;
            int32_t any = 0;
            for (int g = 0; g < es.ng; ++g) any |= f[g];
            if (any == 0) {  // app_{it-1} satisfies every check: converged at it - 1
                if (pos == 0) es.conv[cw] = es.it - 1;
                return;
            }
        }
    }
    const int gend = min(T, (tb + 1) * tpw);
    for (int gi = tb * tpw; gi < gend; ++gi) {
        const int64_t so = (int64_t)cw * t.M;
        if (gi < t.G) {
            const int64_t vo = (int64_t)cw * t.n + (int64_t)gi * kIZ;
            const int d = t.vdeg[gi];
            cint32* row = t.vn + gi * kIVS;
#if IRA_VN_PAIR
            // two information tasks of one degree: both tasks' loads in flight together
            const bool two = gi + 1 < gend && gi + 1 < t.G && t.vdeg[gi + 1] == d;
#endif
            static_for<1, MAXDV + 1>([&](auto DD) __attribute__((always_inline)) {
                constexpr int D = decltype(DD)::value;
                if (d == D) {
#if IRA_VN_PAIR
                    if (two) {
                        VnIn<D> i0, i1;
                        ira_vn_load<D>(row, vo, so, pos, L, S, i0);
                        ira_vn_load<D>(row + kIVS, vo + kIZ, so, pos, L, S, i1);
                        __builtin_amdgcn_sched_barrier(0);
                        ira_vn_sum<D>(row, vo, pos, app, i0);
                        ira_vn_sum<D>(row + kIVS, vo + kIZ, pos, app, i1);
                    } else {
                        ira_vn_info<D>(row, vo, so, pos, L, S, app);
                    }
#else
                    ira_vn_info<D>(row, vo, so, pos, L, S, app);
#endif
                }
            });
#if IRA_VN_PAIR
            gi += two ? 1 : 0;
#endif
        } else if (!IRA_DIAG_NOPAR) {
            // parity p_j, j = r + q pos: checks j (its own (r, pos), slot kIPS) and j + 1 (slot kIPS + 1 there)
            const int r = pgrp > 0 ? min((gi - t.G + 1) * pgrp, t.q) - 1 : gi - t.G;
            const int p = min(pos, kIZ - 1);
            const float a = L[(int64_t)cw * t.n + t.k + (int64_t)r * kIZ + p];
            const int64_t i0 = so + (int64_t)r * kIZ + p;
            int r1 = r + 1, p1 = p;
            if (r1 == t.q) {
                r1 = 0;
                p1 = p + 1;
            }
            const bool has1 = p1 < kIZ;  // j + 1 < M
            const int64_t i1 = so + (int64_t)r1 * kIZ + (has1 ? p1 : 0);
            const IraState s0 = ira_ld_i(S, i0), s1 = ira_ld_i(S, i1);
#if IRA_VN_SCHED
            __builtin_amdgcn_sched_barrier(0);  // both states and L in flight before the first use
#endif
            const float c0 = ira_c2v(s0, kIPS);
            const float x1 = ira_c2v(s1, kIPS + 1);
            const float c1 = has1 ? x1 : -0.0f;  // x + (-0) == x bit for bit: the last parity has one check
            if (pos < kIZ) par.p[(int64_t)cw * par.stride + (int64_t)r * kIZ + pos] = (a + c0) + c1;
        }
    }
}

// One task = one check row a of one codeword; lanes = positions b.  Reads the posteriors of the row's variables
// and its own state, writes the new state (the oracle's k_cn_ms arithmetic on v2c = app - c2v).
// Parity posteriors read from `pr`; with FUSE (IRA_CNPAR) the next iteration's parity posteriors of every row but
// the group's last are written to `pw` (the variable kernel forms the rest), from L (`L`) and the new states.
template <int MAXR, bool FUSE, bool ES>
__global__ __launch_bounds__(kIraLanes) void k_ira_cn(IRADev t, const float* __restrict__ app, ParBuf pr, ParBuf pw,
                                                      const float* __restrict__ L, IraState* __restrict__ S, int Bc,
                                                      float clamp, float alpha, float beta, int tpw, IraEs es) {
    int cw, tb;
    if (!ira_task((t.q + tpw - 1) / tpw, Bc, cw, tb)) return;
    const int pos = threadIdx.x;
    if constexpr (ES) {
        if (es.conv[cw] != 0) return;
    }
    bool unsat = false;  // ES, it >= 1: some check of this lane's rows fails on app_it
    const int p = min(pos, kIZ - 1);
    const float* const prc = pr.p + (int64_t)cw * pr.stride;
    const int64_t ao = (int64_t)cw * t.n;
    const int r0 = tb * tpw, r1 = min(t.q, (tb + 1) * tpw);
    IraState prev = {0.0f, 0.0f, 0u};  // FUSE: the new state of the previous row at this position
    struct In {
        IraState st;
        float ap0, ap1, lp;
        float v[MAXR];
    };
    // every load of row ra: its state, both parity posteriors, L of parity (ra - 1, p) (FUSE) and the gathers
    auto fetch = [&](int ra, In& in) __attribute__((always_inline)) {
        const int64_t si = (int64_t)cw * t.M + (int64_t)ra * kIZ + p;
        const int R = t.cdeg[ra];
        cint32* row = t.cn + ra * kICS;
        in.st = ira_ld_i(S, si);
        in.ap0 = prc[(int64_t)ra * kIZ + p];
        const int64_t pi = ra > 0 ? (int64_t)(ra - 1) * kIZ + p : (int64_t)(t.q - 1) * kIZ + (p > 0 ? p - 1 : 0);
        in.ap1 = prc[pi];
        const bool fuse = FUSE && ra > r0;  // parity (ra - 1, p): both its checks' new states are here
        in.lp = fuse ? L[ao + t.k + (int64_t)(ra - 1) * kIZ + p] : 0.0f;
        // the row's table entries as one scalar load before any use (inside the per-slot branches each entry was
        // its own load and wait, and each slot's posterior load waited on it)
        int ent[MAXR];
        static_for<0, MAXR>([&](auto SS) __attribute__((always_inline)) { ent[decltype(SS)::value] = row[decltype(SS)::value]; });
        static_for<0, MAXR>([&](auto SS) __attribute__((always_inline)) {
            constexpr int s = decltype(SS)::value;
            // MAXR <= 8: every slot loads (a slot past R reads the zero-padded table entry: group 0 at this position,
            // a cache hit, unused), so no load sits in a branch and all of them are in flight before the first wait
            if (MAXR <= 8 || s < R) {
                const int e = ent[s];
                const int g = e & 0xff, sh = e >> 8;
                int m = p - sh;
                m += m < 0 ? kIZ : 0;
                in.v[s] = app[ao + (int64_t)g * kIZ + m];
            }
        });
    };
    auto update = [&](int ra, In& in) __attribute__((always_inline)) {
        const int64_t si = (int64_t)cw * t.M + (int64_t)ra * kIZ + p;
        const int R = t.cdeg[ra];
        const IraState st = in.st;
        const float ap0 = in.ap0, ap1 = in.ap1;
        float* const v = in.v;
        if constexpr (ES) {  // the check on app_it: xor of its variables' decisions (z = app / 2)
            if (es.it >= 1) {
                bool par = Num<float>::bit(0.5f * ap0);
                if (ra > 0 || p > 0) par ^= Num<float>::bit(0.5f * ap1);
                static_for<0, MAXR>([&](auto SS) __attribute__((always_inline)) {
                    constexpr int s = decltype(SS)::value;
                    if (s < R) par ^= Num<float>::bit(0.5f * v[s]);
                });
                unsat |= par && pos < kIZ;
            }
        }
        float min1 = __builtin_inff(), min2 = __builtin_inff();
        int idx = -1;
        uint32_t sgn = 0;
        // branch-free two-minimum (as written with if / else-if the compiler made every slot a divergent branch with
        // exec-mask saves and register shuffles): m < min1 -> (m, min1, s); else min2 = min(min2, m) — the same
        // values, magnitudes being >= +0 and never NaN
        auto take = [&](float x, int s) __attribute__((always_inline)) {
            const float m = fabsf(x);
            sgn ^= f2u(x);
            const bool lt = m < min1;
            min2 = lt ? min1 : fminf(min2, m);
            min1 = lt ? m : min1;
            idx = lt ? s : idx;
        };
        static_for<0, MAXR>([&](auto SS) __attribute__((always_inline)) {
            constexpr int s = decltype(SS)::value;
            if (s < R) {
                v[s] = v[s] - ira_c2v(st, s);
                take(v[s], s);
            }
        });
        const float vp0 = ap0 - ira_c2v(st, kIPS);
        const float vp1 = ap1 - ira_c2v(st, kIPS + 1);
        const bool has_prev = ra > 0 || p > 0;  // check 0 has no p_{-1}
        take(vp0, kIPS);
        if (has_prev) take(vp1, kIPS + 1);
        const float mag1 = ms_mag(min1, alpha, beta, clamp);
        const float mag2 = ms_mag(min2, alpha, beta, clamp);
        uint32_t meta = (uint32_t)idx << 27;
        static_for<0, MAXR>([&](auto SS) __attribute__((always_inline)) {
            constexpr int s = decltype(SS)::value;
            if (s < R) meta |= ((sgn ^ f2u(v[s])) >> 31) << s;
        });
        meta |= ((sgn ^ f2u(vp0)) >> 31) << kIPS;
        if (has_prev) meta |= ((sgn ^ f2u(vp1)) >> 31) << (kIPS + 1);
        const IraState nst{mag1, mag2, meta};
        if (pos < kIZ) ira_st_i(S, si, nst);
        if constexpr (FUSE) {
            if (ra > r0 && pos < kIZ)
                pw.p[(int64_t)cw * pw.stride + (int64_t)(ra - 1) * kIZ + pos] =
                    (in.lp + ira_c2v(prev, kIPS)) + ira_c2v(nst, kIPS + 1);
            prev = nst;
        }
    };
#if IRA_CN_PF
    // software-pipelined: row ra + 1's loads are issued before row ra's arithmetic, so each wave keeps two rows of
    // loads in flight (the kernel runs about one round of workgroups per launch: the loads in flight per wave, not
    // the number of waves, set how much of the memory latency is hidden)
    In cur;
    fetch(r0, cur);
    for (int ra = r0; ra < r1; ++ra) {
        In nxt;
        if (ra + 1 < r1) fetch(ra + 1, nxt);
        __builtin_amdgcn_sched_barrier(0);
        update(ra, cur);
        cur = nxt;
    }
#else
    for (int ra = r0; ra < r1; ++ra) {
        In in;
        fetch(ra, in);
#if IRA_CN_SCHED
        __builtin_amdgcn_sched_barrier(0);  // the state, both parity posteriors, L and every gather in flight first
#endif
        update(ra, in);
    }
#endif
    if constexpr (ES) {  // this group's word (every thread of the workgroup gets here)
        const bool any = __syncthreads_or(unsat || es.it == 0);
        if (threadIdx.x == 0) es.flg[(int64_t)cw * es.ng + tb] = any ? 1 : 0;
    }
}

// natural [B][n] llr -> permuted L = -llr: information part as is, parity block [360][q] (index b*q + a)
// transposed to [q][360] through an LDS tile.  grid: x = tiles of one codeword, y = codeword.
__global__ __launch_bounds__(256) void k_ira_load(const float* __restrict__ llr, float* __restrict__ L, int n, int k,
                                                  int q) {
    __shared__ float tile[64][65];
    const int64_t base = (int64_t)blockIdx.y * n;
    const int ninfo = (k + 1023) / 1024;
    if ((int)blockIdx.x < ninfo) {
        const int v0 = blockIdx.x * 1024;
        for (int v = v0 + threadIdx.x; v < v0 + 1024 && v < k; v += 256) L[base + v] = -llr[base + v];
        return;
    }
    const int tix = blockIdx.x - ninfo;
    const int ta = (q + 63) / 64;
    const int b0 = (tix / ta) * 64, a0 = (tix % ta) * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {  // rows b, columns a: coalesced along a in the natural layout
        const int b = b0 + r, a = a0 + tx;
        if (b < kIZ && a < q) tile[r][tx] = -llr[base + k + (int64_t)b * q + a];
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {  // rows a, columns b: coalesced along b in the permuted layout
        const int a = a0 + r, b = b0 + tx;
        if (b < kIZ && a < q) L[base + k + (int64_t)a * kIZ + b] = tile[tx][r];
    }
}

// z = 0.5 app (the oracle's final layer for min-sum, bp.py:51's decision rule) back to the natural layout:
// bits (np.round(p1) rule) and soft (p1 = 1 - sigmoid(z), or z).
// ES: a converged codeword's posteriors are those of iteration conv[cw]: its parity part is in par[conv & 1];
// iters_used (the chunk's slice, or null) gets conv or iters
__global__ __launch_bounds__(256) void k_ira_out(const float* __restrict__ app, ParBuf p0, ParBuf p1, int iters,
                                                 const int32_t* __restrict__ conv, int32_t* __restrict__ used,
                                                 uint8_t* __restrict__ bits, float* __restrict__ soft, int soft_z, int n,
                                                 int k, int q) {
    const int32_t cu = conv ? conv[blockIdx.y] : 0;
    const int u = cu ? cu : iters;
    const ParBuf par = (u & 1) ? p1 : p0;
    if (used && blockIdx.x == 0 && threadIdx.x == 0) used[blockIdx.y] = u;
    __shared__ float tile[64][65];
    const int64_t base = (int64_t)blockIdx.y * n;
    const int ninfo = (k + 1023) / 1024;
    auto put = [&](int64_t i, float z) __attribute__((always_inline)) {
        if (bits) bits[i] = (uint8_t)Num<float>::bit(z);
        if (soft) soft[i] = soft_z ? z : 1.0f - 1.0f / (1.0f + Num<float>::exp_(-z));
    };
    if ((int)blockIdx.x < ninfo) {
        const int v0 = blockIdx.x * 1024;
        for (int v = v0 + threadIdx.x; v < v0 + 1024 && v < k; v += 256) put(base + v, 0.5f * app[base + v]);
        return;
    }
    const int tix = blockIdx.x - ninfo;
    const int ta = (q + 63) / 64;
    const int b0 = (tix / ta) * 64, a0 = (tix % ta) * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int a = a0 + r, b = b0 + tx;
        if (b < kIZ && a < q) tile[r][tx] = 0.5f * par.p[(int64_t)blockIdx.y * par.stride + (int64_t)a * kIZ + b];
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int b = b0 + r, a = a0 + tx;
        if (b < kIZ && a < q) put(base + k + (int64_t)b * q + a, tile[tx][r]);
    }
}

// ---- host ------------------------------------------------------------------------------------------------

IRASpec* ira_detect(int m, int n, const int32_t* rp, const int32_t* ci, int device) {
    if (m <= 0 || n <= m || m % kIZ || (n - m) % kIZ) return nullptr;
    const int M = m, k = n - m, q = m / kIZ, G = k / kIZ;
    if (q > 255 || G > 255) return nullptr;
    // parity part: row c holds k + c and (c >= 1) k + c - 1, nothing else above k
    std::vector<int32_t> vdeg_all(k, 0);
    for (int c = 0; c < M; ++c) {
        int np = 0;
        bool own = false, prev = false;
        for (int e = rp[c]; e < rp[c + 1]; ++e) {
            const int v = ci[e];
            if (v >= k) {
                ++np;
                own |= v == k + c;
                prev |= c > 0 && v == k + c - 1;
            } else {
                ++vdeg_all[v];
            }
        }
        if (!own || np != (c > 0 ? 2 : 1) || (c > 0 && !prev)) return nullptr;
    }
    // information columns: column lists (ascending checks)
    std::vector<int32_t> cptr(k + 1, 0), cchk;
    for (int v = 0; v < k; ++v) cptr[v + 1] = cptr[v] + vdeg_all[v];
    cchk.resize(cptr[k]);
    {
        std::vector<int32_t> fill(cptr.begin(), cptr.end() - 1);
        for (int c = 0; c < M; ++c)
            for (int e = rp[c]; e < rp[c + 1]; ++e)
                if (ci[e] < k) cchk[fill[ci[e]]++] = c;
    }
    IRASpec* s = new IRASpec();
    s->q = q; s->G = G; s->k = k; s->n = n; s->M = M; s->E = rp[M]; s->device = device;
    std::vector<int32_t> vn((size_t)G * kIVS, 0), vdeg(G, 0), cn((size_t)q * kICS, 0), cdeg(q, 0);
    std::vector<std::vector<std::pair<int, int>>> rows(q);  // (group, shift) per check row
    bool ok = true;
    for (int g = 0; g < G && ok; ++g) {
        const int v0 = g * kIZ;
        const int d = cptr[v0 + 1] - cptr[v0];
        if (d < 1 || d > kIVS) { ok = false; break; }
        std::vector<int> xs(cchk.begin() + cptr[v0], cchk.begin() + cptr[v0 + 1]);  // ascending = the x order
        std::vector<int> want(d);
        for (int mm = 1; mm < kIZ && ok; ++mm) {
            const int v = v0 + mm;
            if (cptr[v + 1] - cptr[v] != d) { ok = false; break; }
            for (int t = 0; t < d; ++t) want[t] = (int)(((int64_t)xs[t] + (int64_t)mm * q) % M);
            std::sort(want.begin(), want.end());
            for (int t = 0; t < d; ++t)
                if (cchk[cptr[v] + t] != want[t]) { ok = false; break; }
        }
        vdeg[g] = d;
        s->maxdv = std::max(s->maxdv, d);
        for (int t = 0; t < d && ok; ++t) {
            const int a = xs[t] % q, sh = xs[t] / q;
            const int slot = (int)rows[a].size();
            if (slot >= kICS) { ok = false; break; }
            rows[a].push_back({g, sh});
            vn[(size_t)g * kIVS + t] = a | (sh << 8) | (slot << 17);
        }
    }
    for (int a = 0; a < q && ok; ++a) {
        cdeg[a] = (int)rows[a].size();
        s->maxr = std::max(s->maxr, cdeg[a]);
        for (int i = 0; i < cdeg[a]; ++i) cn[(size_t)a * kICS + i] = rows[a][i].first | (rows[a][i].second << 8);
    }
    if (!ok) {
        delete s;
        return nullptr;
    }
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != device) (void)hipSetDevice(device);
    auto up = [](int32_t** d, const std::vector<int32_t>& h) -> bool {
        if (hipMalloc((void**)d, h.size() * 4) != hipSuccess) return false;
        return hipMemcpy(*d, h.data(), h.size() * 4, hipMemcpyHostToDevice) == hipSuccess;
    };
    ok = up(&s->vn, vn) && up(&s->vdeg, vdeg) && up(&s->cn, cn) && up(&s->cdeg, cdeg);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    if (!ok) {
        ira_free(s);
        return nullptr;
    }
    return s;
}

void ira_free(IRASpec* s) {
    if (!s) return;
    (void)hipFree(s->vn);
    (void)hipFree(s->vdeg);
    (void)hipFree(s->cn);
    (void)hipFree(s->cdeg);
    delete s;
}

bool ira_supports(const IRASpec* s, const ldpc_params& p) {
    if (!s) return false;
    if (p.algo != LDPC_ALGO_MIN_SUM) return false;
    if (p.flags & LDPC_F_F64) return false;
    if (getenv("LDPC_NO_IRA")) return false;  // A/B against the generic kernels in one process
    return s->maxdv <= 16 && s->maxr <= kICS;
}

// codewords per chunk: the arrays of the chunks in flight (8n + 12M bytes per codeword) stay in the 256 MiB
// Infinity Cache for all their iterations; LDPC_IRA_BUDGET_MB overrides (0 = the whole batch in one pass).  Config
// [4], B = 4,096, one stream (profiles/r05/ab/ab_c4_ira_tpw.txt): 100 MB 28.2k cw/s, 200 MB 32.8k, 240 MB 33.6k,
// 256 MB 34.0k, 400 MB 25.2k; two streams: 200 MB 41.55k, 256 MB 41.3k, 320 MB 35.5k (ab_c4_ira_streams.txt).
// Round 6, after the variable sums without the rotation network and the branch-free check kernel (two streams,
// profiles/r06/ab/ab_c4_ira_vn_cn.txt): 200 MB 59.1k, 230 MB 59.5k, 250 MB 59.7k, 270 MB 46.3k (out of the Infinity
// Cache): 240 shipped, clear of the cliff.
static int64_t ira_chunk(const IRASpec* s, int64_t B, int ns = 1) {
    const char* env = getenv("LDPC_IRA_BUDGET_MB");
    const int64_t budget = ((env ? (int64_t)atol(env) : 240) << 20) / ns;
    if (budget <= 0) return B;
    const int64_t per = 8 * (int64_t)s->n + 12 * (int64_t)s->M + (IRA_CNPAR ? 4 * (int64_t)s->M : 0);
    int64_t bc = budget / per / 8 * 8;
    if (bc < 8) bc = 8;
    if (bc >= B) return B;
    // balanced: the fewest chunks of at most bc codewords, equal sizes (rounded up to 8) — no short last chunk
    // whose launches would leave most of the chip idle
    const int64_t nch = (B + bc - 1) / bc;
    const int64_t eq = ((B + nch - 1) / nch + 7) / 8 * 8;
    return eq < bc ? eq : bc;
}

// chunks decoded side by side on NS streams (the caller's and NS - 1 forked ones), each 1/NS of the budget
// (LDPC_IRA_STREAMS, 1..4).  Two kernels of different chunks fill each other's ramp, drain and latency gaps:
// config [4] 38.3 -> 41.3-41.6k cw/s with 2 streams, 41.6-41.8k with 3, 41.2k with 4
// (profiles/r05/ab/ab_c4_ira_streams.txt); 2 shipped.
static int ira_streams() {
    const char* e = getenv("LDPC_IRA_STREAMS");
    const int v = e ? atoi(e) : 2;
    return v < 1 ? 1 : (v > 4 ? 4 : v);
}

// L, app, check states, (IRA_CNPAR) the second parity-posterior buffer and the early-stop words (conv, flg: at
// most q groups) of bc codewords
static size_t ira_set_bytes(const IRASpec* s, int64_t bc) {
    auto a256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return 2 * a256((size_t)bc * s->n * 4) + a256((size_t)bc * s->M * sizeof(IraState)) +
           (IRA_CNPAR ? a256((size_t)bc * s->M * 4) : 0) + a256((size_t)bc * 4 * (1 + s->q));
}

size_t ira_workspace(const IRASpec* s, int64_t B, const ldpc_params&) {
    const int ns = ira_streams();
    return (size_t)ns * ira_set_bytes(s, ira_chunk(s, B, ns));
}

int ira_decode(const IRASpec* s, const float* llr, int64_t B, const ldpc_params& p, uint8_t* bits, float* soft,
               int32_t* iters_used, char* ws, hipStream_t st) {
    const int ns = ira_streams();
    const int64_t bc = ira_chunk(s, B, ns);
    const size_t set = ira_set_bytes(s, bc);
    auto a256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
    auto cst = [](const int32_t* x) { return (cint32*)x; };  // device tables, written once at graph creation
    const IRADev t{cst(s->vn), cst(s->vdeg), cst(s->cn), cst(s->cdeg), s->q, s->G, s->k, s->n, s->M};
    const int soft_z = (p.flags & LDPC_F_SOFT_Z) ? 1 : 0;
    const unsigned tiles = (unsigned)((s->k + 1023) / 1024 + ((kIZ + 63) / 64) * ((s->q + 63) / 64));
    // tasks per workgroup: one task is a short wave (a few loads, one store); at one task per workgroup a launch is
    // ~40 k short workgroups: 4 tasks took config [4] 28.8k -> 33.0k cw/s (200 MB chunks), 16 tasks 20.8k (too few
    // workgroups) — profiles/r05/ab/ab_c4_ira_tpw.txt
    // per kernel: VN 4, CN 6 (a divisor of q = 90 for DVB-S2 1/2; A/B profiles/r05/ab/ab_c4_ira_tpw_split.txt);
    // LDPC_IRA_TPW sets both, LDPC_IRA_TPW_VN / _CN one
    auto env_int = [](const char* name, int dflt) {
        const char* e = getenv(name);
        return e && atoi(e) > 0 ? atoi(e) : dflt;
    };
    const int tp_all = env_int("LDPC_IRA_TPW", 0);
    const int tpv = env_int("LDPC_IRA_TPW_VN", tp_all ? tp_all : 4);
    const int tpw = env_int("LDPC_IRA_TPW_CN", tp_all ? tp_all : 6);
    hipStream_t str[4] = {st, st, st, st};
    const int nch = (int)((B + bc - 1) / bc);
    const int nf = (ns < nch ? ns : nch) - 1;  // forked streams in use
    if (nf > 0)
        if (const int rc = aux_fork(st, &str[1], nf)) return rc;
    int i = 0;
    for (int64_t o = 0; o < B; o += bc, ++i) {
        const int k = i % (nf + 1);
        hipStream_t q = str[k];
        char* w = ws + (size_t)k * set;
        float* L = (float*)w;
        float* app = (float*)(w + a256((size_t)bc * s->n * 4));
        IraState* S = (IraState*)(w + 2 * a256((size_t)bc * s->n * 4));
        // parity posteriors: P[0] in app's parity region, P[1] its own buffer (IRA_CNPAR; otherwise P[0] again)
        const ParBuf P0{app + s->k, s->n};
        const ParBuf P1 = IRA_CNPAR ? ParBuf{(float*)(w + 2 * a256((size_t)bc * s->n * 4) +
                                                      a256((size_t)bc * s->M * sizeof(IraState))), s->M}
                                    : P0;
        int32_t* esw = (int32_t*)(w + 2 * a256((size_t)bc * s->n * 4) + a256((size_t)bc * s->M * sizeof(IraState)) +
                                  (IRA_CNPAR ? a256((size_t)bc * s->M * 4) : 0));
        const bool es_on = (p.flags & LDPC_F_EARLY_STOP) != 0;
        IraEs es{esw, esw + bc, (s->q + tpw - 1) / tpw, 0};
        const int b = (int)(B - o < bc ? B - o : bc);
        const int64_t vo = o * s->n;
        const unsigned cw8 = (unsigned)((b + 7) / 8) * 8;
        k_ira_load<<<dim3(tiles, b), 256, 0, q>>>(llr + vo, L, s->n, s->k, s->q);
        if (hipMemsetAsync(S, 0, (size_t)b * s->M * sizeof(IraState), q) != hipSuccess)
            return set_error(LDPC_EHIP, "IRA state init failed");
        if (es_on && hipMemsetAsync(es.conv, 0, (size_t)b * 4, q) != hipSuccess)  // (flg: CN(0) writes every word)
            return set_error(LDPC_EHIP, "IRA early-stop init failed");
        const unsigned gcn = cw8 * (unsigned)((s->q + tpw - 1) / tpw);
        for (int it = 0; it <= p.iters; ++it) {
            // VN(it) writes the parity rows the check kernel did not form into P[it & 1] (all of them before the
            // first check pass); CN(it) reads P[it & 1] and forms the next iteration's into P[(it + 1) & 1]
            const ParBuf pv = (it & 1) ? P1 : P0, pn = (it & 1) ? P0 : P1;
            const int pgrp = (IRA_CNPAR && it > 0) ? tpw : 0;
            const int tv = s->G + (pgrp ? (s->q + pgrp - 1) / pgrp : s->q);
            const unsigned gvn = cw8 * (unsigned)((tv + tpv - 1) / tpv);
            es.it = it;
#define IRA_VN(D, E) k_ira_vn<D, E><<<gvn, kIraLanes, 0, q>>>(t, L, app, S, pv, pgrp, b, tpv, es)
#define IRA_CN(R, E) k_ira_cn<R, IRA_CNPAR, E><<<gcn, kIraLanes, 0, q>>>(t, app, pv, pn, L, S, b, p.clamp, p.alpha, p.beta, tpw, es)
            if (s->maxdv <= 8) {
                if (es_on) IRA_VN(8, true); else IRA_VN(8, false);
            } else {
                if (es_on) IRA_VN(16, true); else IRA_VN(16, false);
            }
            if (it == p.iters) break;  // the last VN pass is the final layer's posterior
#if IRA_CN_EXACT
            if (s->maxr <= 5) {
                if (es_on) IRA_CN(5, true); else IRA_CN(5, false);
            } else if (s->maxr <= 6) {
                if (es_on) IRA_CN(6, true); else IRA_CN(6, false);
            } else if (s->maxr <= 8) {
#else
            if (s->maxr <= 8) {
#endif
                if (es_on) IRA_CN(8, true); else IRA_CN(8, false);
            } else {
                if (es_on) IRA_CN(kICS, true); else IRA_CN(kICS, false);
            }
#undef IRA_VN
#undef IRA_CN
        }
        k_ira_out<<<dim3(tiles, b), 256, 0, q>>>(app, P0, P1, p.iters, es_on ? es.conv : nullptr,
                                                 iters_used ? iters_used + o : nullptr, bits ? bits + vo : nullptr,
                                                 soft ? soft + vo : nullptr, soft_z, s->n, s->k, s->q);
    }
    if (nf > 0)
        if (const int rc = aux_join(st, nf)) return rc;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "IRA kernel launch: %s", hipGetErrorString(e));
    return LDPC_OK;
}

}  // namespace ldpc
