// common.h — shared device/host definitions for the gfx950 LDPC decoder.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ldpc_abi.h"

namespace ldpc {

// compile-time loop: f(integral_constant<int, i>) for i in [B, E) — every index a constant, so arrays indexed
// by it stay in registers however large the unrolled body gets (a #pragma unroll can give up)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Hard-decision thresholds: bit = 1 iff np.round(1 - sigmoid(z)) == 1 (ofdm_functions.py:161, bp.py:51).
// fp32: measured bit pattern by bit pattern against torch 2.10 CPU sigmoid -> z <= -1.7881392e-07.
constexpr float kZthrF32 = -1.7881392e-07f;            // 0xb43fffff
constexpr double kZthrF64 = -3.3306690738754696e-16;   // -1.5 * 2^-52 (strict <)
// bp_cv.py:258-261: clamp(p, -(1-eps), 1-eps), eps = 1e-7, the bound cast to the tensor dtype.
constexpr float kPmaxF32 = (float)(1.0 - 1e-7);
constexpr double kPmaxF64 = 1.0 - 1e-7;

// tanh for fp32, restated from the device library's __ocml_tanh_f32 (gfx950 build, ROCm 7.2)
// operation for operation, branch-free and inlinable: the library routine is not inlined into
// kernels built with different IEEE-mode attributes, and as an out-of-line call per edge it cost the
// register-resident tanh-SP kernel a call sequence (and clobbered registers) 88 times per iteration.
//   |x| >= 0.625:  1 - 2 / (1 + 2^(2|x| log2 e))  (exp via v_exp_f32 with a split log2e product)
//   |x| <  0.625:  odd minimax polynomial in x^2
// sign restored with copysign.  Tests compare it with the generic and the oracle paths.
// The library's overflow select (2|x| > 88.72: e = inf) is replaced by clamping 2|x| to 100 before the
// exponential: below 88.72 nothing changes; above it e is >= 2^127 (or inf) either way and the result is
// 1 - 2 / (1 + e) = 1.0 exactly in both forms, so the output bits are the same for every input.
__device__ __forceinline__ float tanh_f32(float x) {
    const float ax = fabsf(x);
    const float t = fminf(ax + ax, 100.0f);
    const float ph = t * 0x1.715476p+0f;                    // 2|x| * log2(e)
    const float n = __builtin_rintf(ph);
    float lo = __builtin_fmaf(t, 0x1.715476p+0f, -ph);
    lo = __builtin_fmaf(t, 0x1.4ae0bep-26f, lo);
    const float f = (ph - n) + lo;
    const float e = __builtin_ldexpf(__builtin_amdgcn_exp2f(f), (int)n);
    const float big = __builtin_fmaf(__builtin_amdgcn_rcpf(1.0f + e), -2.0f, 1.0f);
    const float x2 = x * x;
    float p = __builtin_fmaf(-0x1.758e7ap-8f, x2, 0x1.521192p-6f);
    p = __builtin_fmaf(x2, p, -0x1.b8389cp-5f);
    p = __builtin_fmaf(x2, p, 0x1.110704p-3f);
    p = __builtin_fmaf(x2, p, -0x1.555532p-2f);
    p = ax * p;
    const float small = __builtin_fmaf(x2, p, ax);
    return __builtin_copysignf(t >= 1.25f ? big : small, x);  // t = 2|x| exactly below the clamp
}

// fp32 division n / d as the device library lowers it (v_div_scale, Newton-Raphson on v_rcp_f32,
// v_div_fmas, v_div_fixup) with the scaling and fix-up steps dropped.  For normal operands whose
// exponents differ by far less than 96 — here n, d in [2^-23, 2] — v_div_scale returns its operand,
// v_div_fmas is a plain fma and v_div_fixup the identity, so the bits are the library's (correctly
// rounded) quotient; 8 instead of 11 instructions, none of them VCC-writing (no hazard nops).
__device__ __forceinline__ float div_f32_unscaled(float n, float d) {
    float r = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(-d, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    float q = n * r;
    const float e2 = __builtin_fmaf(-d, q, n);
    q = __builtin_fmaf(e2, r, q);
    const float e3 = __builtin_fmaf(-d, q, n);
    return __builtin_fmaf(e3, r, q);
}

// logf as the device library computes it (__ocml_log_f32: v_log_f32, then log2 -> ln in extended
// precision) for NORMAL finite x: the library's denormal prescale and its inf/nan pass-through select
// never fire there, so this is the same bits in 5 instead of 12 instructions.
__device__ __forceinline__ float log_f32_normal(float x) {
    const float r = __builtin_amdgcn_logf(x);
    const float h = r * 0x1.62e42ep-1f;                 // 0x3f317217
    float lo = __builtin_fmaf(r, 0x1.62e42ep-1f, -h);
    lo = __builtin_fmaf(r, 0x1.efa39ep-25f, lo);        // 0x3377d1cf
    return h + lo;
}

// Check-node output of the tanh rule for one edge (bp_cv.py:44-50, then the caller's clamp, bp.py:47):
// p clamped to +-(1-1e-7), y = log((1+p)/(1-p)), clamped to +-clamp.  The clamps are med3 (same values
// as the two compare-and-set statements for every non-NaN input, -0 included).  fp32: (1+p), (1-p) lie in
// [2^-23, 2] and their quotient in [2^-24, 2^24], so the restated division and logf above are exact
// stand-ins for `/` and logf.
__device__ __forceinline__ float cn_tanh_out(float p, float clamp) {
    p = __builtin_amdgcn_fmed3f(p, -kPmaxF32, kPmaxF32);
    const float y = log_f32_normal(div_f32_unscaled(1.0f + p, 1.0f - p));
    return __builtin_amdgcn_fmed3f(y, -clamp, clamp);
}
__device__ __forceinline__ double cn_tanh_out(double p, double clamp) {
    if (p > kPmaxF64) p = kPmaxF64;
    if (p < -kPmaxF64) p = -kPmaxF64;
    double y = log((1.0 + p) / (1.0 - p));
    if (y > clamp) y = clamp;
    if (y < -clamp) y = -clamp;
    return y;
}

__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float u2f(uint32_t u) { return __uint_as_float(u); }

// ---- fp32 tanh sum-product in the (D, S) form (oracle/ldpc_oracle.c cn_stable_f32) ----------------
// The same function as bp_vc.py:27 + bp.py:29 + bp_cv.py:38-50, evaluated without the reference's
// cancellation near |p| -> 1.  The VC side hands the check a signed a = copysign(exp(-|s|), s), s = L +
// exclusive sum (twice the reference's tanh argument: |tanh(s/2)| = (1-a)/(1+a)).  A set of edges is a pair
// (D, S) ~ (P+ - P-, P+ + P-) with P+- = prod(1 +- a); the identity is (0, 1), one edge adds D' = D + a*S,
// S' = S + a*D (two fma), two sets join as D = Dp*Sq + Sp*Dq, S = Sp*Sq + Dp*Dq (one product and one fma
// each, ds_join_out; an edge with s = +-0, a = 1, keeps D == S exactly through pushes and as a join's suffix,
// to an ulp as its prefix — so such edges are handled explicitly, ds_fix_one).  The check output of an edge is
// log(S/D) of the set of the others (= log((1+|p|)/(1-|p|))), at most log RMAX where RMAX =
// (1+pmax)/(1-pmax) = 16777215 is the reference's fp32 p clamp (bp_cv.py:44-47) exactly, and at most the
// caller's clamp (bp.py:47); its sign the xor of the others' signs.
//
// Messages travel in LOG2 UNITS ("bits"): the fp32 tanh-SP kernels' c2v messages and VC sums are the
// natural-log values times log2(e); L stays -llr.  The VC argument is s2 = fma(L, log2 e, sum2) (one fma, as the
// add it replaces); a = exp2(-|s2|) is one v_exp_f32 with a -|x| source modifier; the check output is
// log2(S/D) — one v_log_f32 — clamped once to [0, cmax2], cmax2 = min(fp32(clamp * log2 e), 24 = fp32(log2
// RMAX)); z = fma(sum2, ln2 / 2, 0.5 * L), exactly 0.5 * L when no message reaches the variable (zero
// iterations).  Natural-log messages cost a multiply on each side (by log2 e before exp2, by ln 2 after log2)
// and a second clamp; the results differ by rounding only (tests/softparity.py holds both to the reference's
// fp64).
constexpr float kRmaxF32 = 16777215.0f;
constexpr float kLog2eF32 = 0x1.715476p+0f;    // fp32(log2 e)
constexpr float kHalfLn2F32 = 0x1.62e430p-2f;  // fp32(ln 2 / 2): z = 0.5 * L-sum in natural units
constexpr float kCeilLog2F32 = 24.0f;          // fp32(log2 16777215)
__device__ __forceinline__ float sp_cmax2(float clamp) { return fminf(clamp * kLog2eF32, kCeilLog2F32); }
// z = 0.5 * (L + sum) with the sum in log2 units (fp32) or natural units (fp64, the reference's operations)
template <typename T> __device__ __forceinline__ T sp_z(T L, T sum) { return T(0.5) * (L + sum); }
template <> __device__ __forceinline__ float sp_z<float>(float L, float sum2) {
    return __builtin_fmaf(sum2, kHalfLn2F32, 0.5f * L);
}
// the VC argument s2 = (L + sum) * log2 e with the sum already in log2 units
__device__ __forceinline__ float sp_vn_arg(float L, float sum2) { return __builtin_fmaf(L, kLog2eF32, sum2); }

// signed a = copysign(exp(-|s|), s) of a VC sum s2 = s * log2 e: one v_exp_f32 of -|s2|.  A relative error of
// ulp(s2) in s2 moves the check output log(S/D) by at most that much absolutely; |s| beyond the clamp saturates.
// DS_CR (diagnostic builds only, scripts/trace_config2.py): bit 0 / 1 / 2 evaluate exp2 / the division S/D / log2
// correctly rounded (through fp64, the oracle's exp2f / S / D / log2f) instead of v_exp_f32 / S * v_rcp_f32(D) /
// v_log_f32, to name the operation that separates the kernels from their specification.  Shipped: 0.
#ifndef DS_CR
#define DS_CR 0
#endif
// DS_DIAG_NOTRANS (DIAGNOSTIC BUILDS ONLY, wrong results): the three transcendentals (v_exp_f32 here, v_rcp_f32 and
// v_log_f32 in ds_out) replaced by one fma each, to price what their issue cost and latency take from a kernel
#ifndef DS_DIAG_NOTRANS
#define DS_DIAG_NOTRANS 0
#endif
__device__ __forceinline__ float vn_signed_a(float x2) {
#if DS_DIAG_NOTRANS
    return __builtin_copysignf(__builtin_fmaf(-fabsf(x2), 0x1p-6f, 1.0f), x2);
#elif DS_CR & 1
    return __builtin_copysignf((float)exp2(-(double)fabsf(x2)), x2);
#else
    return __builtin_copysignf(__builtin_amdgcn_exp2f(-fabsf(x2)), x2);
#endif
}

// SP_TIE(operands): the serial-chain tie of the tanh-SP kernels, an empty asm that redefines the chain's
// values (so the next edge's chain depends on this edge's output).  Its cost: the hazard recognizer takes an
// asm-defined VGPR for a possible transcendental result, so a VALU reading it right after gets an s_nop
// (~100 of the (648,1/2) loop's 231).  SP_TIE_SCHED (a scheduling barrier instead, no operands) spills
// 46 VGPRs there and 287 in the sliced kernel: not used.
#ifndef SP_TIE_SCHED
#define SP_TIE_SCHED 0
#endif
#if SP_TIE_SCHED
#define SP_TIE(...) __builtin_amdgcn_sched_barrier(0)
#else
#define SP_TIE(...) asm volatile("" : __VA_ARGS__)
#endif

// VC exclusive sums of one column of compile-time degree d in O(d) — 3d - 6 adds instead of the ~d^2 / 2 of
// re-summing the others per edge; the oracle's stable form (sp_f32_one) sums in the same order:
// Q_k = x_k + ... + x_{d-1} right to left, P_k = x_0 + ... + x_{k-1} left to right, S_0 = Q_1,
// S_{d-1} = P_{d-1}, S_k = P_k + Q_{k+1} (d = 1: S_0 = +0).  x(k) reads message k, out(k, S_k) runs in k order
// after x(k)'s last read (it may overwrite message k in place).  TIE = t > 0: the running prefix is tied (an
// empty asm) after every t-th output, so one edge's chain is in flight at a time.
template <int d, int TIE, class X, class Out>
__device__ __forceinline__ void vn_excl_sums(X&& x, Out&& out) {
    if constexpr (d == 1) {
        out(std::integral_constant<int, 0>{}, 0.0f);
    } else if constexpr (d > 1) {
        float Q[d];  // Q[k], 1 <= k < d
        Q[d - 1] = x(std::integral_constant<int, d - 1>{});
        static_for<0, d - 2>([&](auto ii) __attribute__((always_inline)) {
            constexpr int k = d - 2 - decltype(ii)::value;
            Q[k] = Q[k + 1] + x(std::integral_constant<int, k>{});
        });
        float P = 0.0f;
        static_for<0, d>([&](auto kk) __attribute__((always_inline)) {
            constexpr int k = decltype(kk)::value;
            float S;
            if constexpr (k == 0) S = Q[1];
            else if constexpr (k == d - 1) S = P;
            else S = P + Q[k + 1];
            if constexpr (k == 0) P = x(kk);
            else if constexpr (k < d - 1) P = P + x(kk);
            out(kk, S);
            if constexpr (TIE > 0 && (k + 1) % TIE == 0) SP_TIE("+v"(P));
        });
    }
}

struct DSet {
    float D, S;
};
__device__ __forceinline__ DSet ds_identity() { return {0.0f, 1.0f}; }
__device__ __forceinline__ DSet ds_push(DSet x, float a) {  // a = |signed a| of one more edge
    return {__builtin_fmaf(a, x.S, x.D), __builtin_fmaf(a, x.D, x.S)};
}
// log2(S/D) of a set clamped to [0, cmax2] (S >= D; a rounding below 1 gives 0; D == 0: +inf -> cmax2), with
// the given sign bit (bit 31 of sgn)
__device__ __forceinline__ float ds_out(float D, float S, uint32_t sgn, float cmax2) {
#if DS_DIAG_NOTRANS
    const float r = __builtin_fmaf(S, 0.5f, D);
#elif DS_CR & 2
    const float r = (float)((double)S / (double)D);  // S, D exact in fp64: one rounding = the oracle's S / D
#else
    const float r = S * __builtin_amdgcn_rcpf(D);
#endif
#if DS_DIAG_NOTRANS
    const float y = __builtin_amdgcn_fmed3f(__builtin_fmaf(r, 0.25f, -1.0f), 0.0f, cmax2);
#elif DS_CR & 4
    const float y = __builtin_amdgcn_fmed3f((float)log2((double)r), 0.0f, cmax2);
#else
    const float y = __builtin_amdgcn_fmed3f(__builtin_amdgcn_logf(r), 0.0f, cmax2);
#endif
    return u2f(f2u(y) | (sgn & 0x80000000u));
}
// the output of an edge from its prefix set p and suffix set q (the join, then ds_out).  DS_JOIN_FMA: each of
// D and S is one product and one fma (D = fma(p.D, q.S, p.S * q.D), S = fma(p.D, q.D, p.S * q.S)), 4 VALU per
// join instead of 6 (two products and an add each); both round at most twice, as before.  A symmetric suffix
// (q.D == q.S: it holds an edge with a = 1, s = +-0) still gives D == S exactly — both are fma(p.D, x, p.S * x)
// — so such an edge zeroes the others' outputs as the reference's p = 0; a symmetric prefix gives D, S within
// an ulp (an output <= 2^-23 in log2 units instead of 0).  The oracle (ldpc_oracle.c cn_stable_f32) joins the same way.
#ifndef DS_JOIN_FMA
#define DS_JOIN_FMA 1
#endif
__device__ __forceinline__ float ds_join_out(DSet p, DSet q, uint32_t sgn, float cmax2) {
#if DS_JOIN_FMA
    const float D = __builtin_fmaf(p.D, q.S, p.S * q.D);
    const float S = __builtin_fmaf(p.D, q.D, p.S * q.S);
#else
    const float D = p.D * q.S + p.S * q.D;  // -ffp-contract=off: two products and one add each
    const float S = p.S * q.S + p.D * q.D;
#endif
    return ds_out(D, S, sgn, cmax2);
}

// One check row of compile-time degree d: g[] holds the gathered signed a of its edges (check frame) and
// receives their outputs.  Suffix sets are built right to left, then a left-to-right pass joins each
// edge's prefix with the suffix after it (edges 0 and d-1 need no join): 2(d-1) + 2(d-1) fma + 4(d-2)
// products/adds.  SERIAL = k > 0 ties every k-th edge's output to the running prefix (an empty asm), so the
// scheduler keeps at most k edges' logs in flight instead of interleaving the whole row's (0: no ties).
#ifndef DS_SPLIT_D
#define DS_SPLIT_D 12  // rows longer than this run in blocks (register budget of the sliced Z = 81 kernel)
#endif
#ifndef DS_BLOCK
#define DS_BLOCK 7  // (1944,5/6) d = 20: 3 blocks, 128 VGPRs spill-free at 4 waves/SIMD (10: 3 VGPRs spilled)
#endif
#ifndef DS_TSHARE
#define DS_TSHARE 1
#endif
// LAG = 1 (with SERIAL = 1): the running prefix after edge t is tied to edge t - 1's output instead of edge t's,
// so edge t's output (rcp, log) overlaps edge t + 1's join — two edges in flight, same operations.
template <int t, int LAG, int d>
__device__ __forceinline__ void ds_tie(DSet& pre, float (&g)[d]) {
    if constexpr (LAG == 0) SP_TIE("+v"(pre.D), "+v"(pre.S), "+v"(g[t]));
    else if constexpr (t >= LAG) SP_TIE("+v"(pre.D), "+v"(pre.S), "+v"(g[t - LAG]));
}
// Edges with a == 1 (s = +-0: the reference's tanh(0) = 0 makes p exactly 0 for every OTHER edge of the check,
// bp_cv.py:38-50): an edge whose exclusive set holds one outputs exactly +-0 (oracle cn_stable_f32).  The (D, S)
// sets give that by themselves except through a join with such a PREFIX (an ulp apart, DS_JOIN_FMA) and S/D
// rounded through v_rcp_f32, and several such edges per check (erasures, quantized LLRs) add up to a flipped
// hard decision (tests/golden/bp_zeros.npz).  cn_ds_row<..., FIX = true> marks the row's a == 1 edges in the low
// bits of the row's sign word (whose bit 31 alone the outputs read, so no register is added) and resets each
// output whose other edges include one to its sign bit as it is formed.
// THE RULE (round 6, one for every kernel and the oracle): it applies to the codewords whose LLRs hold an exact
// zero (+-0) — the source of a == 1 edges: s = 0 needs L = 0 or an exact cancellation — for all their
// iterations; a codeword without one runs the plain form throughout, where an a == 1 edge (an exact
// cancellation, or |s| so small that exp rounds to 1) leaves its partners within 2^-23 (log2 units) of 0.  The
// register kernels run the FIX loop for a wave / unit with such a codeword (fixm masks the lanes of its other
// codeword), the plain loop otherwise; the generic kernels read a flag per codeword (k_load_llr).
#ifndef QC_SP_FIXZ
#define QC_SP_FIXZ 1  // register kernels: the FIX loop for waves / units with an exact-zero LLR (0: never)
#endif
template <int d>
__device__ __forceinline__ uint32_t ds_ones(const float (&g)[d]) {
    uint32_t ones = 0;
    static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
        constexpr int t = decltype(tt)::value;
        ones |= (fabsf(g[t]) == 1.0f ? 1u : 0u) << t;
    });
    return ones;
}
// output y of edge t of a row whose a == 1 edges are marked in bits 0..30 of sgw: +-0 if another edge is marked
template <int t>
__device__ __forceinline__ float ds_fix_one(float y, uint32_t sgw) {
    static_assert(t < 31, "the a == 1 marks share the sign word with its bit 31");
    return (sgw & 0x7fffffffu & ~(1u << t)) ? u2f(f2u(y) & 0x80000000u) : y;
}

// fixm (FIX): 0x7fffffff where the lane's codeword holds an exact-zero LLR, 0 where it does not (the rule is per
// codeword: a lane of a codeword without one keeps the plain outputs, whatever its unit's other codeword has)
template <int d, int SERIAL, int LAG = 0, int BLOCK = DS_BLOCK, bool FIX = false>
__device__ __forceinline__ void cn_ds_row(float (&g)[d], float cmax2, uint32_t fixm = 0x7fffffffu) {
    const float clamp = cmax2;  // (log2 units, sp_cmax2)
    constexpr auto tie_after = [](int t) { return SERIAL > 0 && (t + 1) % SERIAL == 0; };

    // xor of the row's sign words, three at a time (v_bitop3_b32 0x96)
    uint32_t sg = f2u(g[0]);
    static_for<0, (d - 1) / 2>([&](auto pp) __attribute__((always_inline)) {
        constexpr int k = 1 + 2 * decltype(pp)::value;
        sg = __builtin_amdgcn_bitop3_b32(sg, f2u(g[k]), f2u(g[k + 1]), 0x96);
    });
    if constexpr (d % 2 == 0) sg ^= f2u(g[d - 1]);
    if constexpr (FIX && d > 1) sg = (sg & 0x80000000u) | (ds_ones(g) & fixm);  // the row's a == 1 edges (ds_fix_one)
    if constexpr (d == 1) {
        g[0] = ds_out(0.0f, 1.0f, 0u, clamp);  // empty product: p = 1 -> the ceiling, positive
    } else if constexpr (d > DS_SPLIT_D) {
        // Long rows (802.11n 1944 5/6: d = 20) in blocks of DS_BLOCK edges, so only one block's suffix sets
        // are live: per block, the set T of the edges after it (fresh pushes from the row's end), then the
        // block's suffixes from T and its outputs with the running prefix.  Every set is formed by the same
        // pushes in the same order as the unblocked pass, so the outputs are bitwise the unblocked ones; the
        // cost is the T passes.  (Each block's T pushes copies of the inputs through an empty asm: otherwise
        // the compiler CSEs the passes and keeps every suffix set live, which is what blocking avoids.)
        constexpr int BS = BLOCK < d ? BLOCK : d, NBK = (d + BS - 1) / BS;
        DSet pre = {0.0f, 1.0f};
        // DS_TSHARE: one pass from the row's end yields every block's T (the sets at the block boundaries,
        // the same pushes in the same order), instead of a fresh pass per block
        [[maybe_unused]] float TD[NBK], TS[NBK];
        if constexpr (DS_TSHARE) {
            float a = fabsf(g[d - 1]);
            asm volatile("" : "+v"(a));
            DSet T = {a, 1.0f};
            if constexpr ((d - 1) % BS == 0) {  // a block ends at hi = d - 1: its T is the last edge alone
                TD[(d - 1) / BS - 1] = T.D;
                TS[(d - 1) / BS - 1] = T.S;
            }
            static_for<0, d - 1 - BS>([&](auto uu) __attribute__((always_inline)) {
                constexpr int t = d - 2 - decltype(uu)::value;  // d-2 down to BS
                float b = fabsf(g[t]);
                asm volatile("" : "+v"(b));
                T = ds_push(T, b);
                if constexpr (t % BS == 0) {  // t = hi of block t / BS - 1
                    TD[t / BS - 1] = T.D;
                    TS[t / BS - 1] = T.S;
                }
            });
        }
        static_for<0, NBK>([&](auto kk) __attribute__((always_inline)) {
            constexpr int lo = decltype(kk)::value * BS, hi = (lo + BS < d) ? lo + BS : d;
            float sD[BS + 1], sS[BS + 1];  // sD[t - lo]: set of edges t..d-1, lo < t <= hi
            if constexpr (hi < d && DS_TSHARE) {
                sD[hi - lo] = TD[decltype(kk)::value];
                sS[hi - lo] = TS[decltype(kk)::value];
            } else if constexpr (hi < d) {
                float a = fabsf(g[d - 1]);
                asm volatile("" : "+v"(a));
                DSet T = {a, 1.0f};
                static_for<0, d - 1 - hi>([&](auto uu) __attribute__((always_inline)) {
                    float b = fabsf(g[d - 2 - decltype(uu)::value]);
                    asm volatile("" : "+v"(b));
                    T = ds_push(T, b);
                });
                sD[hi - lo] = T.D;
                sS[hi - lo] = T.S;
            }
            static_for<0, hi - lo - 1>([&](auto uu) __attribute__((always_inline)) {
                constexpr int t = hi - 1 - decltype(uu)::value;  // hi-1 down to lo+1
                if constexpr (t == d - 1) {
                    sD[t - lo] = fabsf(g[t]);
                    sS[t - lo] = 1.0f;
                } else {
                    const DSet q = ds_push({sD[t + 1 - lo], sS[t + 1 - lo]}, fabsf(g[t]));
                    sD[t - lo] = q.D;
                    sS[t - lo] = q.S;
                }
            });
            static_for<lo, hi>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                const float a = fabsf(g[t]);
                float y;
                if constexpr (t == 0) y = ds_out(sD[1 - lo], sS[1 - lo], sg ^ f2u(g[t]), clamp);
                else if constexpr (t == d - 1) y = ds_out(pre.D, pre.S, sg ^ f2u(g[t]), clamp);
                else y = ds_join_out(pre, {sD[t + 1 - lo], sS[t + 1 - lo]}, sg ^ f2u(g[t]), clamp);
                if constexpr (FIX) y = ds_fix_one<t>(y, sg);
                if constexpr (t == 0) pre = {a, 1.0f};
                else if constexpr (t < d - 1) pre = ds_push(pre, a);
                g[t] = y;
                if constexpr (tie_after(t)) ds_tie<t, LAG>(pre, g);
            });
        });
    } else {
        float sD[d], sS[d];  // suffix set of edges t..d-1, t >= 1
        sD[d - 1] = fabsf(g[d - 1]);
        sS[d - 1] = 1.0f;
        static_for<0, d - 2>([&](auto kk) __attribute__((always_inline)) {
            constexpr int t = d - 2 - decltype(kk)::value;
            const DSet q = ds_push({sD[t + 1], sS[t + 1]}, fabsf(g[t]));
            sD[t] = q.D;
            sS[t] = q.S;
        });
        DSet pre = {fabsf(g[0]), 1.0f};
        g[0] = ds_out(sD[1], sS[1], sg ^ f2u(g[0]), clamp);
        if constexpr (FIX) g[0] = ds_fix_one<0>(g[0], sg);
        if constexpr (tie_after(0)) SP_TIE("+v"(pre.D), "+v"(g[0]));
        static_for<1, d - 1>([&](auto tt) __attribute__((always_inline)) {
            constexpr int t = decltype(tt)::value;
            const float a = fabsf(g[t]);
            float y = ds_join_out(pre, {sD[t + 1], sS[t + 1]}, sg ^ f2u(g[t]), clamp);
            if constexpr (FIX) y = ds_fix_one<t>(y, sg);
            pre = ds_push(pre, a);
            g[t] = y;
            if constexpr (tie_after(t)) ds_tie<t, LAG>(pre, g);
        });
        g[d - 1] = ds_out(pre.D, pre.S, sg ^ f2u(g[d - 1]), clamp);
        if constexpr (FIX) g[d - 1] = ds_fix_one<d - 1>(g[d - 1], sg);
    }
}

template <typename T> struct Num;
template <> struct Num<float> {
    __device__ static float tanh_(float x) { return tanh_f32(x); }
    __device__ static float exp_(float x) { return expf(x); }
    __device__ static bool bit(float z) { return z <= kZthrF32; }
};
template <> struct Num<double> {
    __device__ static double tanh_(double x) { return tanh(x); }
    __device__ static double exp_(double x) { return exp(x); }
    __device__ static bool bit(double z) { return z < kZthrF64; }
};

// min-sum check-node output magnitude (oracle/ldpc_oracle.c ms_f32_one): min(clamp, max(alpha*m - beta, 0))
__device__ __forceinline__ float ms_mag(float m, float alpha, float beta, float clamp) {
    float x = alpha * m;
    x = fmaxf(x - beta, 0.0f);
    return fminf(x, clamp);
}

// ---- counter-based normal generator (Philox-4x32-10 + Box-Muller) for the on-device channel ----
struct Philox {
    __device__ static void round_(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0, uint32_t k1) {
        const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
        uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
        uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    __device__ static void gen(uint64_t ctr, uint64_t key, uint32_t out[4]) {
        uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0x5bd1e995u, c3 = 0x1b873593u;
        uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            round_(c0, c1, c2, c3, k0, k1);
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
    }
};

}  // namespace ldpc

// internal entry points shared between translation units
namespace ldpc {
int set_error(int code, const char* fmt, ...);
int fill_i32(int32_t* p, int64_t count, int32_t value, hipStream_t st);

struct GenericArgs {
    const int32_t *row_ptr, *col_idx, *var_ptr, *var_edges;
    int m, n, E, max_dc, max_dv;
    const int32_t* wofs;  // [n+1] start of variable v's d_v x d_v block in one iteration's compact VN weights
    int64_t W;            // sum_v d_v^2
};
// Weighted BP (bp_vc.py:16-27 with non-unit weights): device arrays of the decode precision, any may be
// null (= all ones).  vn [iters][W], lw [iters][n], fin [E] (var-slot order), flw [n].
struct BPWeights {
    const void *vn, *lw, *fin, *flw;
    const void* c2v0 = nullptr;  // initial c2v [B][E] check-order (the reference's x, bp/bp.py:43-47); NULL = 0
};
size_t generic_workspace(const GenericArgs& g, int64_t B, const ldpc_params& p);
int generic_decode(const GenericArgs& g, const void* llr_dev, int64_t B, const ldpc_params& p, uint8_t* bits,
                   void* soft, int32_t* iters_used, char* ws, hipStream_t st, const BPWeights* w = nullptr);

// Structure-specialised (quasi-cyclic) decoders compiled into the library (qc.hip).
struct QCSpec;
const QCSpec* qc_lookup(int mb, int nb, int z, const int32_t* shifts);
int qc_z(const QCSpec* s);
bool qc_supports(const QCSpec* s, const ldpc_params& p);
size_t qc_workspace(const QCSpec* s, int64_t B, const ldpc_params& p);
int qc_decode(const QCSpec* s, const void* llr_dev, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
              int32_t* iters_used, char* ws, hipStream_t st);

// tanh-SP register kernels, two passes (qc.hip k_qc_sp_st, qc_sl_sp.h): qc_sp_fork zeroes the list, runs
// k_sp_zero_scan on st (the waves / units whose LLRs hold an exact zero: [0] = count, [1 .. B] ids, then one flag
// byte per unit, in the decode's workspace) and forks a second stream from it; the a == 1 rule's pass walks the
// list on that stream while the plain pass (which skips flagged units) runs on st; qc_sp_join joins them.
// qc_decode sets the workspace pointer for the launchers it calls on this host thread.
uint32_t*& qc_sp_zlist();
__host__ __device__ inline uint8_t* qc_sp_zflag(uint32_t* zlist, int64_t B) {
    return reinterpret_cast<uint8_t*>(zlist + 1 + B);
}
int qc_sp_fork(const float* llr, int64_t B, int n, int cpu, hipStream_t st, hipStream_t* s2);
int qc_sp_join(hipStream_t st);
// up to 3 extra streams per (host thread, device, caller stream), forked from / joined back into the caller's stream
// by events (graph-capturable); one fork / join pair at a time per caller stream and thread (qc.hip)
int aux_fork(hipStream_t st, hipStream_t* s2, int n = 1);
int aux_join(hipStream_t st, int n = 1);
constexpr unsigned kSpPass2Blocks = 1280;  // second-pass grid cap: 5 units per CU
inline unsigned qc_sp_pass2_grid(unsigned blocks) { return blocks < kSpPass2Blocks ? blocks : kSpPass2Blocks; }

// IRA codes with the DVB-S2 structure (Z = 360), min-sum (ira.hip)
struct IRASpec;
IRASpec* ira_detect(int m, int n, const int32_t* row_ptr, const int32_t* col_idx, int device);
void ira_free(IRASpec* s);
bool ira_supports(const IRASpec* s, const ldpc_params& p);
size_t ira_workspace(const IRASpec* s, int64_t B, const ldpc_params& p);
int ira_decode(const IRASpec* s, const float* llr, int64_t B, const ldpc_params& p, uint8_t* bits, float* soft,
               int32_t* iters_used, char* ws, hipStream_t st);
}  // namespace ldpc
