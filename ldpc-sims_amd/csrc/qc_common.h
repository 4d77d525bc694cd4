// qc_common.h — compile-time helpers shared by the quasi-cyclic register kernels (qc.hip, qc_sl.hip).
#pragma once
#include "common.h"
#include "qc_tables.h"

#include <type_traits>

namespace ldpc {

// first block row whose checks touch block column j (VN adds start there, so L_j is read there)
template <class C>
constexpr int first_row(int j) {
    for (int r = 0; r < C::MB; ++r)
        for (int t = 0; t < C::DEG[r]; ++t)
            if (C::COL[r][t] == j) return r;
    return -1;
}
template <class C>
constexpr int first_slot(int r, int j) {
    for (int t = 0; t < C::DEG[r]; ++t)
        if (C::COL[r][t] == j) return t;
    return -1;
}

// ms_mag (oracle: min(clamp, max(alpha*m - beta, 0))) specialised on which of alpha != 1 / beta != 0
// hold: alpha == 1 makes alpha*m exact and beta == 0 makes max(m - 0, 0) == m for m >= 0 (m is a
// minimum of |v|, never negative), so each form is bit-identical to the general one for its case.
enum { NORM_PLAIN = 0, NORM_ALPHA = 1, NORM_BETA = 2, NORM_BOTH = 3 };
template <int NORM>
__device__ __forceinline__ float mag_of(float m, float alpha, float beta, float clamp) {
    if constexpr (NORM == NORM_PLAIN) return fminf(m, clamp);
    else if constexpr (NORM == NORM_ALPHA) return fminf(alpha * m, clamp);
    else if constexpr (NORM == NORM_BETA) return fminf(fmaxf(m - beta, 0.0f), clamp);
    else return ms_mag(m, alpha, beta, clamp);
}

// The two smallest |v[t]| of a check (multiset order statistics, so any evaluation order gives the same
// values bit for bit).  Three at a time, then pairs: second(S + {x, y}) = min(mn2, med3(mn1, x, y)), so
// each pair costs min3 + med3 + min instead of 2 x (med3 + min): fewer code bytes in a loop bound by
// instruction fetch.  Finite inputs only (no-NaN compile).
template <int D>
__device__ __forceinline__ void two_min(const float (&v)[D], float& mn1, float& mn2) {
    if constexpr (D == 1) {
        mn1 = fabsf(v[0]);
        mn2 = __builtin_inff();
    } else if constexpr (D == 2) {
        mn1 = fminf(fabsf(v[0]), fabsf(v[1]));
        mn2 = fmaxf(fabsf(v[0]), fabsf(v[1]));
    } else {
        mn1 = fminf(fminf(fabsf(v[0]), fabsf(v[1])), fabsf(v[2]));
        mn2 = __builtin_amdgcn_fmed3f(fabsf(v[0]), fabsf(v[1]), fabsf(v[2]));
        static_for<0, (D - 3) / 2>([&](auto pp) __attribute__((always_inline)) {
            constexpr int t = 3 + 2 * decltype(pp)::value;
            const float x = fabsf(v[t]), y = fabsf(v[t + 1]);
            mn2 = fminf(mn2, __builtin_amdgcn_fmed3f(mn1, x, y));
            mn1 = fminf(fminf(mn1, x), y);
        });
        if constexpr ((D - 3) % 2) {
            const float x = fabsf(v[D - 1]);
            mn2 = __builtin_amdgcn_fmed3f(mn1, x, mn2);
            mn1 = fminf(mn1, x);
        }
    }
}

// Lane-major L rows for the register kernels: each lane keeps its NB values of L (or a parked APP) in
// its own LDS row of lstr() floats, columns ordered by the block row that first needs them
// (first_row, ties by column), so one ds_read_b128 brings four columns that are consumed together
// (6 instead of 20-24 LDS reads per iteration at NB = 24).  lstr / 4 is odd: the 16-byte rows of
// 8 consecutive lanes cover disjoint banks (conflict-free b128 reads).
// The orders are tabulated once per code (static constexpr members are evaluated once; the kernels
// query them thousands of times at compile time).
template <class C>
struct LOrder {
    struct Tab {
        int pos[64], col[64];
    };
    static constexpr Tab make() {
        Tab t{};
        int fr[64] = {};
        for (int j = 0; j < C::NB; ++j) fr[j] = first_row<C>(j);
        for (int p = 0; p < 64; ++p) t.col[p] = -1;
        for (int j = 0; j < C::NB; ++j) {
            int p = 0;
            for (int q = 0; q < C::NB; ++q) p += (fr[q] < fr[j]) || (fr[q] == fr[j] && q < j);
            t.pos[j] = p;
            t.col[p] = j;
        }
        return t;
    }
    static constexpr Tab T = make();
};
template <class C>
constexpr int lpos(int j) {
    return LOrder<C>::T.pos[j];
}
template <class C>
constexpr int lcol(int p) {
    return LOrder<C>::T.col[p];
}
template <class C>
constexpr int lstr() {
    const int s = (C::NB + 3) / 4 * 4;
    return ((s / 4) % 2) ? s : s + 4;
}
template <class C>
constexpr int lgroup_row(int g) {  // block row at which group g (positions 4g..4g+3) is first needed
    return first_row<C>(lcol<C>(4 * g));
}

// XOR of the bit patterns of v[0..D) (the sign of a check's product is its bit 31): three inputs per
// v_bitop3_b32 (truth table 0x96), half the VALU instructions of a v_xor chain.
template <int D>
__device__ __forceinline__ uint32_t xor_all(const float (&v)[D]) {
    uint32_t t = __float_as_uint(v[0]);
    static_for<0, (D - 1) / 2>([&](auto pp) __attribute__((always_inline)) {
        constexpr int k = 1 + 2 * decltype(pp)::value;
        t = __builtin_amdgcn_bitop3_b32(t, __float_as_uint(v[k]), __float_as_uint(v[k + 1]), 0x96);
    });
    if constexpr ((D - 1) % 2) t ^= __float_as_uint(v[D - 1]);
    return t;
}

template <class C>
constexpr int edge_off(int r) {
    int o = 0;
    for (int q = 0; q < r; ++q) o += C::DEG[q];
    return o;
}

template <class C>
constexpr int edge_row(int e) {  // block row of (check-order) edge e
    int r = 0;
    while (r + 1 < C::MB && edge_off<C>(r + 1) <= e) ++r;
    return r;
}

template <class C>
constexpr int col_deg(int j) {
    int d = 0;
    for (int r = 0; r < C::MB; ++r)
        for (int t = 0; t < C::DEG[r]; ++t) d += (C::COL[r][t] == j);
    return d;
}
template <class C>
constexpr int col_edge(int j, int k) {  // k-th edge of block column j in ascending row order
    int c = 0;
    for (int r = 0; r < C::MB; ++r)
        for (int t = 0; t < C::DEG[r]; ++t)
            if (C::COL[r][t] == j) {
                if (c == k) return edge_off<C>(r) + t;
                ++c;
            }
    return -1;
}

// ---- lane rotations (ds_bpermute) shared by the register kernels ----------------------------------
#ifndef QC_DIAG_DPP
#define QC_DIAG_DPP 0
#endif
#ifndef QC_DIAG_NOSEL
#define QC_DIAG_NOSEL 0
#endif

// lanes whose lifting index z lies in [lo, hi), in each codeword's lane group
template <int Z, int CPW>
constexpr uint64_t lane_range_mask(int lo, int hi) {
    uint64_t m = 0;
    for (int z = lo; z < hi; ++z) {
        m |= 1ull << z;
        if (CPW == 2) m |= 1ull << (32 + z);
    }
    return m;
}

// Which lane's slot an idle lane (z >= Z) reads in a rotation.  ds_bpermute and ds_read_b32 serve a wave in
// two 32-lane halves with bank = (address / 4) mod 32; an identical address within a half is a broadcast, a
// second distinct address on a bank one extra LDS cycle.  With one codeword per wave (CPW == 1, 32 < Z < 64)
// the idle lanes 54..63 of Z = 54 sit in the upper half; aliased to lifting index z - Z (round 2) they read
// lanes just above 0..9's sources — a distinct address on a bank the wrapped active lanes use, exactly one
// extra cycle per rotation on every (1296,2/3) rotation (modelled: 104 of 104; measured SQ_LDS_BANK_CONFLICT
// = SQ_INSTS_LDS).  QC_IDLE_ALIAS: alias them to an active lane of the SAME half instead (z' = 32 + (z - Z)
// mod (Z - 32)), wrap decision included, so they repeat its address exactly: 0.62 extra cycles per rotation
// (the rest are the active lanes' own wrap collisions).  CPW == 2 (Z <= 32) is conflict-free either way.
#ifndef QC_IDLE_ALIAS
#define QC_IDLE_ALIAS 1
#endif
template <int Z, int CPW>
constexpr int idle_alias(int z) {  // z >= Z: the lifting index whose rotation addresses this idle lane repeats
    if constexpr (QC_IDLE_ALIAS && CPW == 1 && Z > 32) return 32 + (z - Z) % (Z - 32);
    else return z - Z;
}
template <int Z, int CPW>
__device__ __forceinline__ int lane_zb(int z) {
    return (z < Z) ? z : idle_alias<Z, CPW>(z);
}
// lanes that take the wrapped address of a rotation whose source z + rho reaches Z: z in [lo, Z), and idle
// lanes whose alias is
template <int Z, int CPW>
constexpr uint64_t wrap_mask(int lo) {
    uint64_t m = lane_range_mask<Z, CPW>(lo, Z);
    if (CPW == 1)
        for (int l = Z; l < 64; ++l) {
            const int a = idle_alias<Z, CPW>(l);
            if (a >= lo && a < Z) m |= 1ull << l;
        }
    return m;
}

// lane in MASK ? b : a.  The mask is a compile-time SGPR-pair constant, so the select is one VALU op
// with no v_cmp (and no VCC hazard).  Volatile: never CSE'd across rows or hoisted out of the loop.
//
// A mask whose upper 33 bits are all ones (the sign extension of a negative 32-bit value: e.g. lanes 19..63 of
// a Z = 54 wrap mask with aliased idle lanes) is materialised by the ROCm 7.2 compiler as
// `s_mov_b64 s[..], <32-bit literal>`, which the gfx950 SALU ZERO-extends (measured: every (1296,2/3)
// register kernel decoded garbage; the compiler itself emits `s_mov_b64 s[..], 0xffffffff` for the 64-bit
// value 0x00000000ffffffff elsewhere).  Such masks are passed complemented, with the operands swapped: the
// complement's upper bits are zero, a value either extension reads the same.  tests/test_kernel_resources.py
// checks the built code for 64-bit SALU moves of high-bit literals.
template <uint64_t MASK>
__device__ __forceinline__ int sel_lanes(int a, int b) {
#if QC_DIAG_NOSEL
    (void)b;  // DIAGNOSTIC BUILD ONLY (wrong results): no wrap select, to price the address selects
    return a;
#else
    int r;
    if constexpr ((MASK >> 31) == 0x1FFFFFFFFull)
        asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(~MASK));
    else
        asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(MASK));
    return r;
#endif
}

__device__ __forceinline__ float bperm(int addr, float v) {
#if QC_DIAG_DPP
    // DIAGNOSTIC BUILD ONLY (wrong results): a VALU DPP move instead of the LDS-pipe permute, to price
    // the ds_bpermute traffic.  The address stays live so its computation is still timed.
    asm volatile("" ::"v"(addr));
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xf, 0xf, false));
#else
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
#endif
}

// Lane-mask rotation for the early-stop syndrome: bit i of the result = bit (i + S) mod Z of x, in each
// codeword's lane group (CPW == 2: two 27-bit groups at bits 0 and 32).  Wave-uniform: scalar ALU.
// Bits outside the groups are garbage; the caller masks once per row.
template <int Z, int CPW, int S>
__device__ __forceinline__ uint64_t rot_lanes(uint64_t x) {
    if constexpr (S == 0) {
        return x;
    } else if constexpr (CPW == 1) {
        return (x >> S) ^ (x << (Z - S));
    } else {
        const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
        return ((uint64_t)((hi >> S) ^ (hi << (Z - S))) << 32) | (uint32_t)((lo >> S) ^ (lo << (Z - S)));
    }
}

template <class C>
constexpr int rot_uses(int rho) {  // ds_bpermutes per iteration that read lane (z + rho) mod Z
    int n = 0;
    for (int r = 0; r < C::MB; ++r)
        for (int t = 0; t < C::DEG[r]; ++t) {
            const int s = C::SHR[r][t];
            n += (s != 0 && (s == rho || C::Z - s == rho));
        }
    return n;
}

// An LDS element re-read at every use instead of hoisted into a register across the iteration loop (register
// budget): `boff` is this lane's byte offset, made opaque per use; OFF (bytes, a compile-time constant) rides in
// the instruction's immediate offset.  One v_mov per reload, where an opaque element index cost a v_mov and a
// v_lshlrev (the index * 4) per reload.
template <int OFF, class T, int ALIGN = alignof(T)>
__device__ __forceinline__ T lds_reload(const void* base, int boff) {
    asm volatile("" : "+v"(boff));
    const char* p = reinterpret_cast<const char*>(base) + boff + OFF;
    return *static_cast<const T*>(__builtin_assume_aligned(p, ALIGN));
}

}  // namespace ldpc
