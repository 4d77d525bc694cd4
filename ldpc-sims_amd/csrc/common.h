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

__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float u2f(uint32_t u) { return __uint_as_float(u); }

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
}  // namespace ldpc
