// qc_pk.hip — quantized (integer offset) min-sum for the 802.11n QC codes with Z <= 64: TWO codewords per
// lane, packed as an fp16 pair in every register.
//
// The quantized decoder's values are small integers: LLRs and messages in [-qmax, qmax] (qmax <= 127),
// posteriors L + sum c2v in [-(1 + d_v) qmax, (1 + d_v) qmax] before the app_max clamp — at most 1651 for the
// 802.11n column degrees (<= 12), inside fp16's exact-integer range (2048).  So fp16 arithmetic on them is
// exact and equals the oracle's int arithmetic (oracle/ldpc_oracle.c qms_one) operation for operation, and
// one v_pk_* instruction advances two codewords.  The lane rotations (ds_bpermute, the LDS pipe that bounds
// the float kernels) move 32 bits per lane, i.e. both codewords at once: half the LDS traffic per codeword.
//
// Structure: k_qc_ms_ph's phased flooding iteration (qc.hip) —
//   CN phase, row by row: v2c (variable frame) gathered into the check frame in place; |v| by masking the
//     two sign bits; the two smallest magnitudes; the sign product; c2v in the check frame.
//   VN phase, column by column: c2v rotated back; APP_j = sat(L_j + sum c2v, app_max); v2c = sat(APP_j - c2v,
//     qmax) for the next iteration.
// Check-node output without a compare (every |v| >= mn1, magnitudes are non-negative and +0 only):
//   min(|v|, mn2) is mn1 for the argmin slot and mn2 for every other slot (ties: mn1 == mn2), so XOR-ing it
//   with mn1 ^ mn2 yields the OTHER minimum bit for bit; offset beta is applied to |v| first,
//   max(|v| - beta, 0), which is monotone, so the order statistics of the offset magnitudes are the offset
//   order statistics (oracle: mag = max(min - beta, 0)).  A -0 v2c (the sign of a zero) changes only the sign
//   of zero-magnitude outputs, so every value equals the oracle's.
// Lane layout: lane (half, z) of wave w holds lifting index z of codewords 2(w*CPW + half) (low fp16) and
// 2(w*CPW + half) + 1 (high), CPW = 2 for Z <= 32 (lane halves), else 1.  The lane frames (PHI) and the
// rotation tables are qc_tables.h's, as in the float kernels.
#include "qc_common.h"

#include <cstdint>

namespace ldpc {

// QC_PK_LDSROT(_EARLY): lane rotations through a per-wave LDS row instead of ds_bpermute (as qc.hip's
// QC_PH_LDSROT).  Off: this kernel is not bound by the LDS pipe — A/B 1-3 % slower in every configuration
// ((1296,2/3) 20 it fixed 50.5 vs 49.8, early stop 49.1 vs 48.4; (648,1/2) 103 vs 102, 101 vs 98 M cw/s).
#ifndef QC_PK_LDSROT
#define QC_PK_LDSROT 0
#endif
#ifndef QC_PK_LDSROT_EARLY
#define QC_PK_LDSROT_EARLY 0
#endif
// QC_PK_DROT(_EARLY): lane rotations through a per-wave DOUBLED LDS row: every active lane stores its value at
// slots z and z + Z of its lane group's row with one ds_write2_b32, and reads slot z + rho (< 2Z: no wrap, so no
// per-rotation address select and no address registers — the offset is the ds immediate); idle lanes write and
// read a private dummy stretch.  A wave's LDS operations run in order, so the row needs no barrier.  Bitwise the
// same results (every packed / quantized parity test passes on it) with 84 fewer VALU per wave-iteration, but
// slower: config [3] 67.3 -> 62.1 M cw/s, fixed count 53.5 -> 50.8, (648,1/2) early stop 114.7 -> 107.9 (A/B
// profiles/r04/ab/ab_drot.txt) — a rotation's store-then-load round trip sits on the chain ds_bpermute shortens.
#ifndef QC_PK_DROT
#define QC_PK_DROT 0
#endif
#ifndef QC_PK_DROT_EARLY
#define QC_PK_DROT_EARLY 0
#endif
#ifndef QC_PK_WAVES_PER_SIMD
#define QC_PK_WAVES_PER_SIMD 4
#endif
#ifndef QC_PK_WAVES_PER_SIMD_EARLY
#define QC_PK_WAVES_PER_SIMD_EARLY 3
#endif
#ifndef QC_PK_ADDR_MIN_USES
#define QC_PK_ADDR_MIN_USES 3  // Z <= 32: rotations used this often per iteration keep their address in a register
#endif
#ifndef QC_PK_ADDR_MIN_USES_Z64
#define QC_PK_ADDR_MIN_USES_Z64 4  // Z > 32 (one lane group): 6 address registers at 4 uses (18 at 3)
#endif
#ifndef QC_PK_ES_ROWS
#define QC_PK_ES_ROWS 1  // early-stop syndrome row by row with an early exit (one codeword pair per wave, Z = 54)
#endif
#ifndef QC_PK_MASK_IDLE
#define QC_PK_MASK_IDLE 0  // A/B -2 % on config [3] (profiles/r04/ab/ab_mask.txt)
#endif
#ifndef QC_PK_DIAG
// DIAGNOSTIC BUILDS ONLY (wrong results; DESIGN.md §3.3, scripts/pk_floor_diag.sh): 1 = no bit stores, 2 = no
// LLR loads — prices the per-launch data movement
#define QC_PK_DIAG 0
#endif
#ifndef QC_PK_PRIO
// 1: s_setprio 1 over the VN phase (0 over the CN phase), early stop and fixed count: config [3] 66.9 -> 67.5 M
// cw/s (A/B profiles/r04/ab/ab_prio.txt); 2: the reverse (-1.3 %)
#define QC_PK_PRIO 1
#endif
#ifndef QC_PK_TPB
#define QC_PK_TPB 256
#endif
// early stop: one-wave workgroups (a workgroup's LDS is held until its slowest wave exits); A/B
// profiles/r02/ab/ab_tpb.txt: config [3] 49.0 -> 50.7 M cw/s (128: 50.1); fixed count: 256 / 128 / 64 equal
#ifndef QC_PK_TPB_EARLY
#define QC_PK_TPB_EARLY 64
#endif
template <bool EARLY>
constexpr int pk_tpb() { return EARLY ? QC_PK_TPB_EARLY : QC_PK_TPB; }

// QC_PK_ILV (one codeword pair per wave, even Z: (1296,2/3), config [3]): lifting index z lives in lane
// (z & 1) * 32 + z / 2 — even z in the lower half, odd in the upper — instead of lane z.  ds_bpermute serves a
// wave in two 32-lane halves with bank = source lane mod 32; with z in lane z every rotation whose source window
// wraps past Z puts two sources of one half on a bank (round 4: SQ_LDS_BANK_CONFLICT 19 % of the kernel's LDS
// cycles).  Interleaved, a rotation by rho = 2v + f reads, for the half of parity e, the half of parity e ^ f at
// lane index (u + v + f e) mod Z/2: distinct lanes of one half, so every rotation is conflict-free.  The early-stop
// ballots are permuted the same way (ilv_rot).  A relabelling of lanes: bitwise the same results.  Off by default:
// measured 2 % slower on config [3] (round 5, profiles/r05/ab): the conflicts it removes were not on the critical
// path, and the interleaved addressing costs VALU in the rotation and epilogue.
#ifndef QC_PK_ILV
#define QC_PK_ILV 0
#endif
template <int Z>
constexpr int ilv_u(int l) {  // a lane's index within its half; an idle lane (index >= Z/2) that of the lane it aliases
    return (l & 31) < Z / 2 ? (l & 31) : ((l & 31) - Z / 2) % (Z / 2);
}
template <int Z>
constexpr uint64_t ilv_active() {
    uint64_t m = 0;
    for (int l = 0; l < 64; ++l) m |= ((l & 31) < Z / 2 ? 1ull : 0ull) << l;
    return m;
}
// lanes whose source lane index of rotation RHO passes Z/2 (they take the wrapped address)
template <int Z, int RHO>
constexpr uint64_t ilv_wrap_mask() {
    uint64_t m = 0;
    for (int l = 0; l < 64; ++l) {
        const int e = l >> 5, u = ilv_u<Z>(l);
        if (u + (RHO >> 1) + ((RHO & 1) ? e : 0) >= Z / 2) m |= 1ull << l;
    }
    return m;
}
// bit l of the result = bit lane((z(l) + S) mod Z) of x (the interleaved counterpart of qc_common.h rot_lanes):
// an even S rotates each half's Z/2-bit field by S/2; an odd S swaps the halves, the lower (even z) taking the
// upper field rotated by (S-1)/2 and the upper the lower rotated by (S+1)/2.  Bits outside the fields: garbage.
template <int Z, int S>
__device__ __forceinline__ uint64_t ilv_rot(uint64_t x) {
    constexpr int H = Z / 2;
    auto r = [](uint32_t y, int k) { return k == 0 ? y : ((y >> k) | (y << (H - k))); };
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if constexpr (S == 0) return x;
    else if constexpr (S % 2 == 0) return ((uint64_t)r(hi, S / 2) << 32) | r(lo, S / 2);
    else return ((uint64_t)r(lo, (S + 1) / 2 % H) << 32) | r(hi, S / 2);
}

using h2 = _Float16 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2 as_h2(uint32_t x) { return __builtin_bit_cast(h2, x); }
__device__ __forceinline__ uint32_t as_u(h2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t pmin(uint32_t a, uint32_t b) { return as_u(__builtin_elementwise_min(as_h2(a), as_h2(b))); }
__device__ __forceinline__ uint32_t pmax(uint32_t a, uint32_t b) { return as_u(__builtin_elementwise_max(as_h2(a), as_h2(b))); }
__device__ __forceinline__ uint32_t padd(uint32_t a, uint32_t b) { return as_u(as_h2(a) + as_h2(b)); }
__device__ __forceinline__ uint32_t psub(uint32_t a, uint32_t b) { return as_u(as_h2(a) - as_h2(b)); }
__device__ __forceinline__ uint32_t pbperm(int addr, uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v); }
__device__ __forceinline__ uint32_t pk2(float lo, float hi) { return as_u(h2{(_Float16)lo, (_Float16)hi}); }
constexpr uint32_t kSign2 = 0x80008000u, kMag2 = 0x7fff7fffu;

template <class C>
constexpr int max_col_deg() {
    int m = 0;
    for (int j = 0; j < C::NB; ++j) m = col_deg<C>(j) > m ? col_deg<C>(j) : m;
    return m;
}
template <class C>
constexpr int min_row_deg() {
    int m = 1 << 30;
    for (int r = 0; r < C::MB; ++r) m = C::DEG[r] < m ? C::DEG[r] : m;
    return m;
}

// three-input packed minimum (v_pk_minimum3_f16, gfx950): IEEE minimum, the same as min on these operands
// (no NaN; magnitudes carry +0 only)
__device__ __forceinline__ uint32_t pmin3(uint32_t a, uint32_t b, uint32_t c) {
    return as_u(__builtin_elementwise_minimum(__builtin_elementwise_minimum(as_h2(a), as_h2(b)), as_h2(c)));
}
#ifndef QC_PK_MIN3
#define QC_PK_MIN3 1  // two-minimum over edge pairs with v_pk_minimum3_f16: 5 VALU per 2 edges instead of 6
#endif
// the two smallest of D packed non-negative magnitudes (each result is one of the inputs, bit for bit).
// QC_PK_MIN3, per pair (x, y) with lo/hi = min/max(x, y): the new second minimum of {mn1 <= mn2, x, y} is
// min(mn2, hi, max(mn1, lo)) (lo < mn1: min(mn1, hi); else min(mn2, lo)), the new minimum min(mn1, lo).
template <int D>
__device__ __forceinline__ void two_min_pk(const uint32_t (&a)[D], uint32_t& mn1, uint32_t& mn2) {
    static_assert(D >= 2, "packed min-sum: check degree >= 2");
    mn1 = pmin(a[0], a[1]);
    mn2 = pmax(a[0], a[1]);
    if constexpr (QC_PK_MIN3) {
        static_for<0, (D - 2) / 2>([&](auto pp) __attribute__((always_inline)) {
            constexpr int t = 2 + 2 * decltype(pp)::value;
            const uint32_t lo = pmin(a[t], a[t + 1]), hi = pmax(a[t], a[t + 1]);
            mn2 = pmin3(mn2, hi, pmax(mn1, lo));
            mn1 = pmin(mn1, lo);
        });
        if constexpr (D % 2 == 1) {
            mn2 = pmin(mn2, pmax(mn1, a[D - 1]));
            mn1 = pmin(mn1, a[D - 1]);
        }
    } else {
        static_for<2, D>([&](auto tt) __attribute__((always_inline)) {
            constexpr int t = decltype(tt)::value;
            mn2 = pmin(mn2, pmax(mn1, a[t]));
            mn1 = pmin(mn1, a[t]);
        });
    }
}

template <int D>
__device__ __forceinline__ uint32_t xor_all_u(const uint32_t (&v)[D]) {
    uint32_t t = v[0];
    static_for<0, (D - 1) / 2>([&](auto pp) __attribute__((always_inline)) {
        constexpr int k = 1 + 2 * decltype(pp)::value;
        t = __builtin_amdgcn_bitop3_b32(t, v[k], v[k + 1], 0x96);
    });
    if constexpr ((D - 1) % 2) t ^= v[D - 1];
    return t;
}

// QC_PK_PAIRS (A/B knob, early stop; default 1): each wave decodes this many codeword pairs one after the other,
// the body straight-line per pair (no runtime loop around it: round 5's persistent loop had raised the register
// demand past the 3-waves/SIMD budget), wave w taking pairs w, w + W, ... (W = the grid's waves)
#ifndef QC_PK_PAIRS
#define QC_PK_PAIRS 1
#endif
template <class C, bool EARLY, bool BETA>
__device__ __forceinline__ void qms_pk_pair(int64_t wave, const float* __restrict__ llr, int64_t B, int iters, float qmax,
                                            float app_max, float beta, float qinv, int flags, uint8_t* __restrict__ bits,
                                            float* __restrict__ soft, int32_t* __restrict__ iters_used, int64_t pair_off) {
    // the work-item id through an empty asm: every lane-derived value is recomputed per pair (QC_PK_PAIRS > 1)
    // rather than kept live from one pair's body into the next
    unsigned tx = threadIdx.x;
    asm volatile("" : "+v"(tx));
    constexpr int Z = C::Z, NB = C::NB, MB = C::MB, N = NB * Z;
    constexpr int NE = edge_off<C>(MB);
    static_assert(Z <= 64, "packed kernel: one lane group per codeword pair");
    static_assert((1 + max_col_deg<C>()) * 127 < 2048, "fp16 must hold every posterior exactly");
    static_assert(min_row_deg<C>() >= 2, "check degree >= 2");
    constexpr int CPW = (Z <= 32) ? 2 : 1;
    constexpr bool LDSROT = EARLY ? QC_PK_LDSROT_EARLY : QC_PK_LDSROT;
    constexpr bool DROT = EARLY ? QC_PK_DROT_EARLY : QC_PK_DROT;
    constexpr bool ILV = QC_PK_ILV && CPW == 1 && Z % 2 == 0 && !LDSROT && !DROT;
    const int lane = tx & 63;
    const int half = (CPW == 2) ? (lane >> 5) : 0;
    // lifting index of this lane (>= Z: idle); ILV: even z in the lower half, odd in the upper
    const int z = ILV ? ((lane & 31) < Z / 2 ? 2 * (lane & 31) + (lane >> 5) : Z + (lane & 31)) : ((CPW == 2) ? (lane & 31) : lane);
    const int64_t cw0 = (wave * CPW + half) * 2;  // low fp16: cw0, high: cw0 + 1
    const int zb = lane_zb<Z, CPW>(z);
    const int base4 = (half * 32 + zb) * 4;
    const int base4m = base4 - 4 * Z;
    // ILV rotation bases: even rotations read this half at index u + v, odd ones the other half at u + e + v
    const int ue = ILV ? 32 * (lane >> 5) + ((lane & 31) < Z / 2 ? (lane & 31) : ((lane & 31) - Z / 2) % (Z / 2)) : 0;
    const int bE = 4 * ue, bO = 4 * ((ue ^ 32) + (lane >> 5));
    using f4 = __attribute__((ext_vector_type(4))) float;
    constexpr int LSTR = lstr<C>();
    __shared__ __attribute__((aligned(16))) uint32_t Ls[pk_tpb<EARLY>() * LSTR];  // lane-major packed L rows (lpos)
    const int lrow = tx * LSTR;
    const int lrow4 = lrow * 4;  // bytes (lds_reload)

    // lane rotations through a per-wave LDS row (as k_qc_ms_ph, qc.hip QC_PH_LDSROT) or ds_bpermute
    __shared__ uint32_t Rw[LDSROT ? pk_tpb<EARLY>() : 1];
    const int wrow = LDSROT ? (int)(tx & ~63u) * 4 : 0;
    const int rb4 = base4 + wrow, rb4m = base4m + wrow;
    if constexpr (LDSROT) {  // M0 = this wave's row, once (nothing else here uses M0); s_nop 0: M0 -> add-TID hazard
        const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(&Rw[0]) + (unsigned)wrow);
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" ::"s"(m0) : "memory");
    }
    auto xfer = [&](int addr, uint32_t x) __attribute__((always_inline)) {
        if constexpr (LDSROT) {
            asm volatile("ds_write_addtid_b32 %0" ::"v"(x) : "memory");
            return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(Rw) + addr);
        } else {
            return pbperm(addr, x);
        }
    };
    constexpr int MINU = (Z <= 32) ? QC_PK_ADDR_MIN_USES : QC_PK_ADDR_MIN_USES_Z64;
    // byte address of "the value of lifting index (z + rho) mod Z" for ds_bpermute
    auto raddr = [&](auto rr) __attribute__((always_inline)) {
        constexpr int rho = decltype(rr)::value;
        if constexpr (ILV) {
            constexpr int v = rho >> 1;
            if constexpr (rho & 1) return sel_lanes<ilv_wrap_mask<Z, rho>()>(bO, bO - 2 * Z) + 4 * v;
            else return sel_lanes<ilv_wrap_mask<Z, rho>()>(bE, bE - 2 * Z) + 4 * v;
        } else {
            return sel_lanes<wrap_mask<Z, CPW>(Z - rho)>(rb4, rb4m) + 4 * rho;
        }
    };
    int ra[Z];
    static_for<1, Z>([&](auto rr) __attribute__((always_inline)) {
        constexpr int rho = decltype(rr)::value;
        if constexpr (rot_uses<C>(rho) >= MINU && !DROT) ra[rho] = raddr(rr);
    });
    constexpr int DW = CPW * 2 * Z + 64 + 2 * Z;  // words per wave: doubled rows, then the idle lanes' stretch
    __shared__ uint32_t Rd[DROT ? (pk_tpb<EARLY>() / 64) * DW : 1];
    const int da = DROT ? 4 * ((int)(tx >> 6) * DW + ((z < Z) ? half * 2 * Z + z : CPW * 2 * Z + lane)) : 0;
    auto rot = [&](auto rr, uint32_t x) __attribute__((always_inline)) {  // value of lane (z + rho) mod Z
        constexpr int rho = decltype(rr)::value;
        if constexpr (rho == 0) {
            return x;
        } else if constexpr (DROT) {
            static_assert(4 * Z <= 255 * 4, "ds_write2 offset1 is 8 bits (in dwords)");
            asm volatile("ds_write2_b32 %0, %1, %1 offset1:%2" ::"v"((unsigned)(uintptr_t)&Rd[0] + (unsigned)da), "v"(x),
                         "i"(Z)
                         : "memory");
            return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(Rd) + da + 4 * rho);
        } else if constexpr (rot_uses<C>(rho) >= MINU) {
            return xfer(ra[rho], x);
        } else {
            return xfer(raddr(rr), x);
        }
    };
    (void)ra;

    // packed constants (SGPRs)
    const uint32_t QM = pk2(qmax, qmax), NQM = pk2(-qmax, -qmax), AM = pk2(app_max, app_max), NAM = pk2(-app_max, -app_max);
    const uint32_t BT = pk2(beta, beta);

    // L = -sat(rint(llr / qstep), qmax) of both codewords (the float kernels' quantizer, in fp32), packed into
    // this lane's LDS row; APP_0 = sat(L, app_max); v2c of iteration 0 = sat(APP_0 - 0, qmax)
    uint32_t msg[NE];
    {
        const bool v0 = (z < Z) && (cw0 < B), v1 = (z < Z) && (cw0 + 1 < B);
        uint32_t L[NB];
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            int t = z + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            const int64_t o = (int64_t)j * Z + t;
#if QC_PK_DIAG == 2  // DIAGNOSTIC BUILD ONLY (wrong results): no LLR loads, to price them
            const float x0 = v0 ? (float)((z * 7 + j) % 9) - 4.0f : 0.0f;
            const float x1 = v1 ? (float)((z * 5 + j) % 9) - 4.0f : 0.0f;
            (void)o;
#else
            const float x0 = v0 ? llr[cw0 * N + o] : 0.0f;
            const float x1 = v1 ? llr[(cw0 + 1) * N + o] : 0.0f;
#endif
            const float q0 = fminf(fmaxf(rintf(x0 * qinv), -qmax), qmax);
            const float q1 = fminf(fmaxf(rintf(x1 * qinv), -qmax), qmax);
            L[j] = pk2(-q0, -q1);
            Ls[lrow + lpos<C>(j)] = L[j];
            L[j] = pmin(pmax(L[j], NAM), AM);
        });
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                msg[edge_off<C>(r) + t] = pmin(pmax(L[C::COL[r][t]], NQM), QM);
            });
        });
    }

    // CN phase: v2c (variable frame) -> c2v (check frame), in place
    auto cn_phase = [&]() __attribute__((always_inline)) {
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            constexpr int e0 = edge_off<C>(r);
            uint32_t v[d], a[d];
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                v[t] = rot(std::integral_constant<int, C::SHR[r][t]>{}, msg[e0 + t]);
                a[t] = v[t] & kMag2;
                if constexpr (BETA) a[t] = pmax(psub(a[t], BT), 0u);  // max(|v| - beta, 0)
            });
            uint32_t mn1, mn2;
            two_min_pk(a, mn1, mn2);
            const uint32_t X = mn1 ^ mn2 ^ (xor_all_u(v) & kSign2);  // sign product folded in
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                const uint32_t other = X ^ pmin(a[t], mn2);
                msg[e0 + t] = __builtin_amdgcn_bitop3_b32(other, v[t], kSign2, 0x78);  // other ^ (v & sign)
            });
        });
    };
    // VN phase, column j: c2v back to the variable frame, APP_j = sat(L_j + sum c2v, app_max)
    f4 Lg;
    auto vn_col = [&](auto pp) __attribute__((always_inline)) {
        constexpr int p = decltype(pp)::value;
        constexpr int j = lcol<C>(p);
        constexpr int dj = col_deg<C>(j);
        if constexpr (p % 4 == 0) {
            Lg = lds_reload<4 * p, f4, 16>(Ls, lrow4);  // not hoisted out of the loop (register budget)
        }
        uint32_t s = __float_as_uint(Lg[p % 4]);
        static_for<0, dj>([&](auto kk) __attribute__((always_inline)) {
            constexpr int e = col_edge<C>(j, decltype(kk)::value);
            constexpr int r = edge_row<C>(e), t = e - edge_off<C>(r);
            constexpr int sh = C::SHR[r][t];
            msg[e] = rot(std::integral_constant<int, (sh == 0) ? 0 : Z - sh>{}, msg[e]);
            s = padd(s, msg[e]);
        });
        return pmin(pmax(s, NAM), AM);
    };
    auto v2c_col = [&](auto jj, uint32_t ap) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) {
            constexpr int e = col_edge<C>(j, decltype(kk)::value);
            msg[e] = pmin(pmax(psub(ap, msg[e]), NQM), QM);
        });
    };

    // early stop: codeword k of this wave = (group g, fp16 half p), k = 2g + p; converged ones park APP
    constexpr uint64_t ACTIVE = ILV ? ilv_active<Z>() : lane_range_mask<Z, CPW>(0, Z);
    constexpr uint64_t G0 = ILV ? ilv_active<Z>() : lane_range_mask<Z, 1>(0, Z), G1 = (CPW == 2) ? (G0 << 32) : 0;
    auto lrot = [&](auto ss, uint64_t b) __attribute__((always_inline)) {  // lane-mask rotation (early stop)
        constexpr int S = decltype(ss)::value;
        if constexpr (ILV) return ilv_rot<Z, S>(b);
        else return rot_lanes<Z, CPW, S>(b);
    };
    constexpr uint32_t ALL = (CPW == 2) ? 0xfu : 0x3u;
    uint32_t done = 0;  // bit k: codeword k converged
    int used0 = iters, used1 = iters, used2 = iters, used3 = iters;
    _Float16* Lh = reinterpret_cast<_Float16*>(Ls);

    int it = 0;
    // QC_PK_MASK_IDLE: idle lanes (z >= Z) sit the iteration loop out, EXEC-masked (as qc.hip QC_PH_MASK_IDLE); the
    // early-stop decisions come from ballots restricted to the active lanes, so they are unchanged
    const bool loop_lane = !QC_PK_MASK_IDLE || z < Z;
    if (loop_lane)
    for (; it + 1 < iters; ++it) {
        if constexpr (QC_PK_PRIO == 1) __builtin_amdgcn_s_setprio(0);
        if constexpr (QC_PK_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        cn_phase();
        if constexpr (QC_PK_PRIO == 1) __builtin_amdgcn_s_setprio(1);
        if constexpr (QC_PK_PRIO == 2) __builtin_amdgcn_s_setprio(0);
        if constexpr (EARLY) {
            uint32_t app[NB];
            static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
                constexpr int p = decltype(pp)::value;
                app[lcol<C>(p)] = vn_col(pp);
            });
            // syndrome of APP_{it+1}: bit 2g + k of `conv` = codeword k (fp16 half) of lane group g satisfies
            // every check.  Per block column one ballot of the hard decisions (oracle: bit = APP < 0) per half,
            // rotated into the frame of each row it touches and XOR-ed there.
            uint32_t conv;
            if constexpr (QC_PK_ES_ROWS && CPW == 1) {
                // Row by row with an early exit (one codeword pair per wave, (1296,2/3)): `conv` starts as the
                // codewords not yet done and loses each one whose row parity is nonzero; the scan stops once no
                // codeword of the wave can still be satisfied — at low Eb/N0 after the first row, so the test
                // costs about one row of scalar rotations instead of all MB.  The ballot is re-taken at every
                // use (one v_cmp): holding 2 x NB of them spilled SGPRs.  The decision is unchanged.
                conv = ALL & ~done;
                static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                    constexpr int r = decltype(rr)::value;
                    if (conv) {
                        static_for<0, 2>([&](auto kk) __attribute__((always_inline)) {
                            constexpr int k = decltype(kk)::value;
                            uint64_t par = 0;
                            static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                                constexpr int t = decltype(tt)::value;
                                const uint64_t b = __ballot(as_h2(app[C::COL[r][t]])[k] < (_Float16)0) & ACTIVE;
                                par ^= lrot(std::integral_constant<int, C::SHR[r][t]>{}, b);
                            });
                            if (par & G0) conv &= ~(1u << k);
                        });
                    }
                });
            } else {  // all rows at once (two codeword pairs per wave: the row-wise form spills 49 VGPRs there)
                conv = 0;
                static_for<0, 2>([&](auto kk) __attribute__((always_inline)) {
                    constexpr int k = decltype(kk)::value;
                    uint64_t par[MB];
#pragma unroll
                    for (int r = 0; r < MB; ++r) par[r] = 0;
                    static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                        constexpr int j = decltype(jj)::value;
                        const uint64_t b = __ballot(as_h2(app[j])[k] < (_Float16)0) & ACTIVE;
                        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                            constexpr int r = decltype(rr)::value;
                            constexpr int t = first_slot<C>(r, j);
                            if constexpr (t >= 0) par[r] ^= lrot(std::integral_constant<int, C::SHR[r][t]>{}, b);
                        });
                    });
                    uint64_t u = 0;
#pragma unroll
                    for (int r = 0; r < MB; ++r) u |= par[r];
                    conv |= ((u & G0) ? 0u : 1u) << k;
                    if constexpr (CPW == 2) conv |= ((u & G1) ? 0u : 1u) << (2 + k);
                });
            }
            const uint32_t fresh = conv & ~done;
            if (fresh) {
                if (fresh & 1u) used0 = it + 1;
                if (fresh & 2u) used1 = it + 1;
                if (fresh & 4u) used2 = it + 1;
                if (fresh & 8u) used3 = it + 1;
                // park APP of a newly converged codeword in its fp16 half of the L row (L no longer needed)
                const int g = (CPW == 2) ? half : 0;
                const bool park0 = (fresh >> (2 * g)) & 1u, park1 = (fresh >> (2 * g + 1)) & 1u;
                if (park0 || park1) {
                    static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                        constexpr int j = decltype(jj)::value;
                        const h2 hv = as_h2(app[j]);
                        if (park0) Lh[2 * (lrow + lpos<C>(j))] = hv[0];
                        if (park1) Lh[2 * (lrow + lpos<C>(j)) + 1] = hv[1];
                    });
                }
                done |= fresh;
                if (done == ALL) break;
            }
            static_for<0, NB>([&](auto jj) __attribute__((always_inline)) { v2c_col(jj, app[decltype(jj)::value]); });
        } else {
            static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
                constexpr int p = decltype(pp)::value;
                v2c_col(std::integral_constant<int, lcol<C>(p)>{}, vn_col(pp));
            });
        }
    }
    // last iteration (or early exit): outputs straight from the VN phase
    const bool early_exit = EARLY && done == ALL;
    if (!early_exit && iters > 0) cn_phase();
    int tid = tx;
    asm volatile("" : "+v"(tid));
    const int zo = ILV ? ((tid & 31) < Z / 2 ? 2 * (tid & 31) + ((tid >> 5) & 1) : Z + (tid & 31))
                       : ((CPW == 2) ? (tid & 31) : (tid & 63));
    const int go = (CPW == 2) ? ((tid >> 5) & 1) : 0;
    const int64_t c0 = (((((int64_t)blockIdx.x * blockDim.x + tid) >> 6) + pair_off) * CPW + go) * 2;
    const bool park0 = EARLY && ((done >> (2 * go)) & 1u), park1 = EARLY && ((done >> (2 * go + 1)) & 1u);
    const bool ok0 = zo < Z && c0 < B, ok1 = zo < Z && c0 + 1 < B;
    static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
        constexpr int p = decltype(pp)::value;
        constexpr int j = lcol<C>(p);
        uint32_t ap;
        if (iters > 0 && !early_exit) ap = vn_col(pp);
        else ap = pmin(pmax(Ls[lrow + p], NAM), AM);  // iters == 0: APP_0; early exit: parked (already sat)
        h2 hv = as_h2(ap);
        if (park0) hv[0] = Lh[2 * (lrow + p)];
        if (park1) hv[1] = Lh[2 * (lrow + p) + 1];
        int t = zo + C::PHI[j];
        t -= (t >= Z) ? Z : 0;
        const int64_t o = (int64_t)j * Z + t;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (k == 0 ? ok0 : ok1) {
                const int64_t oo = (c0 + k) * N + o;
                const float zz = 0.5f * (float)hv[k];
                if (bits && QC_PK_DIAG != 1) bits[oo] = (uint8_t)(zz <= kZthrF32);  // DIAG 1: no output, to price it
                if (soft) soft[oo] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + expf(-zz));
            }
        }
    });
    if (zo == 0 && iters_used) {
        if (ok0) iters_used[c0] = go ? used2 : used0;
        if (ok1) iters_used[c0 + 1] = go ? used3 : used1;
    }
}

template <class C, bool EARLY, bool BETA>
__global__ __launch_bounds__(QC_PK_TPB, EARLY ? QC_PK_WAVES_PER_SIMD_EARLY : QC_PK_WAVES_PER_SIMD) void k_qc_qms_pk(
    const float* __restrict__ llr, int64_t B, int iters, float qmax, float app_max, float beta, float qinv, int flags,
    uint8_t* __restrict__ bits, float* __restrict__ soft, int32_t* __restrict__ iters_used) {
    constexpr int P = EARLY ? QC_PK_PAIRS : 1;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t W = (int64_t)gridDim.x * (blockDim.x >> 6);
    static_for<0, P>([&](auto kk) __attribute__((always_inline)) {
        constexpr int k = decltype(kk)::value;
        qms_pk_pair<C, EARLY, BETA>(wave + k * W, llr, B, iters, qmax, app_max, beta, qinv, flags, bits, soft, iters_used,
                                    k * W);
    });
}

template <class C>
static int launch_qms_pk(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft, int32_t* used,
                         hipStream_t st) {
    constexpr int CPW = (C::Z <= 32) ? 2 : 1;
    const bool es = (p.flags & LDPC_F_EARLY_STOP) != 0;
    const int64_t waves = ((B + 2 * CPW - 1) / (2 * CPW) + (es ? QC_PK_PAIRS : 1) - 1) / (es ? QC_PK_PAIRS : 1);
    const float qm = (float)p.qmax, am = (float)p.app_max, b = p.beta, qi = 1.0f / p.qstep;
    const int tpb = es ? pk_tpb<true>() : pk_tpb<false>();
    const unsigned blocks = (unsigned)((waves + tpb / 64 - 1) / (tpb / 64));
    const float* x = (const float*)llr;
    float* sf = (float*)soft;
#define PK(E, BT) k_qc_qms_pk<C, E, BT><<<blocks, tpb, 0, st>>>(x, B, p.iters, qm, am, b, qi, p.flags, bits, sf, used)
    if (b != 0.0f) {
        if (es) PK(true, true); else PK(false, true);
    } else {
        if (es) PK(true, false); else PK(false, false);
    }
#undef PK
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "qc packed kernel launch: %s", hipGetErrorString(e));
    return LDPC_OK;
}

int qc_launch_qms_pk_wifi648_12(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                                int32_t* used, hipStream_t st) {
    return launch_qms_pk<Wifi648_12>(llr, B, p, bits, soft, used, st);
}
int qc_launch_qms_pk_wifi1296_23(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                                 int32_t* used, hipStream_t st) {
    return launch_qms_pk<Wifi1296_23>(llr, B, p, bits, soft, used, st);
}

}  // namespace ldpc
