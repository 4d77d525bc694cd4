// qc.hip — structure-specialised quasi-cyclic (802.11n) min-sum decoder for gfx950.
//
// One wave decodes CPW codewords entirely in registers for all iterations — one launch per batch, no
// message traffic to HBM (only LLRs in, bits/soft out):
//   * lane <-> lifting index z:  lane (half, z) owns variable (j, z) of every block column j (posterior
//     APP[j] in a VGPR array indexed by compile-time j) and check (r, z) of every block row r (its
//     compressed min-sum state: |c2v| of the min edge and of the others, the argmin slot, and the sign
//     of each outgoing c2v message).  Z <= 32: two codewords per wave (lane halves); Z <= 64: one.
//   * a circulant with shift s connects check (r, i) to variable (j, (i+s) mod Z), so both directions
//     of the exchange are lane rotations inside the codeword's lane group: ds_bpermute_b32 with a
//     2-instruction address (select between two lane-constant bases, shift folded into an immediate);
//     s == 0 circulants need no exchange at all.
//   * the graph is a compile-time constant (qc_tables.h), so every table lookup, loop bound and
//     register index is resolved at compile time.
// Arithmetic is exactly the oracle's (oracle/ldpc_oracle.c ms_f32_one / qms_one): flooding schedule,
// v2c = APP - c2v_old, APP_new = L + sum c2v in ascending check order, same tie rules, same
// normalisation/offset/clamp sequence, same hard-decision rule; so bits and soft outputs are bit-exact.
// Early stop: the syndrome of APP_it is evaluated for free on the values the next iteration's CN
// gathers anyway; a codeword whose syndrome is zero is emitted with iters_used = it.
#include "common.h"
#include "qc_tables.h"

#include <type_traits>

namespace ldpc {

#ifndef QC_ADDR_SGPR_MASK
#define QC_ADDR_SGPR_MASK 1  // rotation-address select with a compile-time lane mask (1 VALU, no v_cmp)
#endif
#ifndef QC_ID_AT_VN
#define QC_ID_AT_VN 1  // find the min slot by |v| == min1 at VN time instead of tracking it in CN
#endif
#ifndef QC_DIAG_DPP
#define QC_DIAG_DPP 0
#endif
#ifndef QC_ROW_BARRIER
#define QC_ROW_BARRIER 0  // measured +1.9% without the per-row scheduling barrier
#endif
#ifndef QC_WAVES_PER_SIMD
#define QC_WAVES_PER_SIMD 5  // 96 VGPRs: 20 waves (40 codewords at Z=27) resident per CU
#endif
#ifndef QC_WAVES_PER_SIMD_EARLY
#define QC_WAVES_PER_SIMD_EARLY 4  // early stop keeps APP_it live to the iteration end: 128 VGPRs
#endif

struct QCSpec {
    int mb, nb, z;
    const int* col;  // [mb][maxdc]
    const int* sh;
    const int* deg;
    int maxdc;
    const char* name;
    int (*launch_ms)(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft, int32_t* used,
                     hipStream_t st);
};

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

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

// lane in MASK ? b : a.  The mask is a compile-time SGPR-pair constant, so the select is one VALU op
// with no v_cmp (and no VCC hazard).  Volatile: never CSE'd across rows or hoisted out of the loop.
template <uint64_t MASK>
__device__ __forceinline__ int sel_lanes(int a, int b) {
    int r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(MASK));
    return r;
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

// QUANT = false: float min-sum.  QUANT = true: integer offset min-sum carried in float registers (all
// values are small integers, so every add/sub is exact and equals the oracle's int arithmetic).
template <class C, bool QUANT, bool EARLY, int NORM>
__global__ __launch_bounds__(256, EARLY ? QC_WAVES_PER_SIMD_EARLY : QC_WAVES_PER_SIMD) void k_qc_ms(const float* __restrict__ llr, int64_t B, int iters, float clamp,
                                               float alpha, float beta, float qmax, float app_max, float qinv,
                                               int flags, uint8_t* __restrict__ bits, float* __restrict__ soft,
                                               int32_t* __restrict__ iters_used) {
    constexpr int Z = C::Z, NB = C::NB, MB = C::MB, N = NB * Z;
    static_assert(Z <= 64, "register kernel needs Z <= 64");
    constexpr int CPW = (Z <= 32) ? 2 : 1;
    const int lane = threadIdx.x & 63;
    const int half = (CPW == 2) ? (lane >> 5) : 0;
    const int z = (CPW == 2) ? (lane & 31) : lane;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t cw = wave * CPW + half;
    const bool valid = (z < Z) && (cw < B);
    // Rotation bases.  Idle lanes (z >= Z) borrow the bases of lane z - Z of their group: their
    // ds_bpermute sources then either coincide with an active lane's source (LDS broadcast) or fall on
    // banks no active lane uses; with their own bases they caused ~1.7 bank-conflict cycles per
    // bpermute (SQ_LDS_BANK_CONFLICT).
    const int zb = (z < Z) ? z : z - Z;
    const int base4 = (half * 32 + zb) * 4;
    const int base4m = base4 - 4 * Z;
    // invalid lanes read element 0 (B >= 1) and discard it: unconditional loads, no per-load branches
    const float* lp = llr + (valid ? cw * N + z : 0);
    const float vmask = valid ? 1.0f : 0.0f;
    constexpr bool early = EARLY;

    // channel LLRs L = -llr (quantized in QUANT mode) staged once in LDS: [wave][half][j][z]
    __shared__ float Ls[4 * CPW * N];
    const int lbase = ((threadIdx.x >> 6) * CPW + half) * N + z;
    float app[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        float x = lp[j * Z] * vmask;
        if (QUANT) x = fminf(fmaxf(rintf(x * qinv), -qmax), qmax);
        app[j] = -x;  // APP before iteration 0 = L + sum(c2v = 0)
        if (z < Z) Ls[lbase + j * Z] = app[j];
    }
    if (QUANT) {
#pragma unroll
        for (int j = 0; j < NB; ++j) app[j] = fminf(fmaxf(app[j], -app_max), app_max);
    }
    float mag1[MB], mag2[MB];
    uint32_t pk[MB];  // bits 0..d-1: sign of c2v slot t at bit (d-1-t); bits 27..31: argmin slot
#pragma unroll
    for (int r = 0; r < MB; ++r) {
        mag1[r] = 0.0f;
        mag2[r] = 0.0f;
        pk[r] = 0u;
    }
    // lanes of this codeword (for the early-stop vote)
    const uint64_t grp = (CPW == 2) ? (((1ull << Z) - 1ull) << (32 * half)) : ((Z == 64) ? ~0ull : ((1ull << Z) - 1ull));
    bool done = !valid;  // per-lane copy of the codeword's state
    int used = iters;
    // bit(z = 0.5*APP) <=> APP <= 2*ZTHR (exact power-of-two scaling)
    const float thr2n = __uint_as_float(__float_as_uint(2.0f * kZthrF32) - 1u);  // negative: -1 ulp = toward +inf

    bool running = true;  // false once every codeword of the wave has converged (early stop)
    for (int it = 0; it < iters && running; ++it) {
        float nap[NB];  // APP_{it+1} = L + sum of new c2v; L_j is read from LDS in the first row touching j
        uint64_t unsat = 0;  // checks (lanes) whose parity over APP_it is odd
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            // Row boundary: fresh (opaque) lane constants stop GVN/LICM from keeping equal-shift rotation
            // addresses of different rows (and iterations) alive; the scheduling barrier keeps those
            // copies inside their row instead of at the loop head.
#if QC_ROW_BARRIER
            __builtin_amdgcn_sched_barrier(0);
#endif
#if QC_ADDR_SGPR_MASK
            // the volatile sel_lanes asm already keeps addresses per row; only the LDS base of the L
            // reloads must be opaque (else LICM hoists the loop-invariant LDS loads: +24 VGPRs)
            const int br = base4, bmr = base4m;
            int lr = lbase;
            asm volatile("" : "+v"(lr));
#else
            int zr = z, br = base4, bmr = base4m, lr = lbase;
            asm volatile("" : "+v"(zr), "+v"(br), "+v"(bmr), "+v"(lr));
#endif
            static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                constexpr int j = decltype(jj)::value;
                if constexpr (first_row<C>(j) == r) nap[j] = Ls[lr + j * Z];
            });
            const uint32_t idx_old = pk[r] >> 27;
            float v[d];
            float mn1 = __builtin_inff(), mn2 = __builtin_inff();
            uint32_t id = 0, tot = 0;
            uint32_t par = 0;  // bit 31 = parity of the hard decisions of this check's variables
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int j = C::COL[r][t], s = C::SH[r][t];
                float a;
                if constexpr (s == 0) {
                    a = app[j];
                } else {
#if QC_ADDR_SGPR_MASK
                    const int addr = sel_lanes<lane_range_mask<Z, CPW>(Z - s, Z)>(br, bmr) + 4 * s;
#else
                    const int addr = ((zr >= Z - s) ? bmr : br) + 4 * s;
#endif
                    a = bperm(addr, app[j]);
                }
                // hard bit(APP) = APP <= thr2 <=> APP - thr2n < 0, thr2n = next float above thr2: a
                // difference of distinct floats is never 0 and never changes sign (denormals kept)
                if constexpr (early) par ^= __float_as_uint(a - thr2n);
                const float om = (idx_old == (uint32_t)t) ? mag2[r] : mag1[r];
                const float old = __uint_as_float(__float_as_uint(om) | ((pk[r] << (31 - (d - 1 - t))) & 0x80000000u));
                float x = a - old;
                if constexpr (QUANT) x = fminf(fmaxf(x, -qmax), qmax);
                v[t] = x;
                const float m = fabsf(x);
#if !QC_ID_AT_VN
                id = (m < mn1) ? (uint32_t)t : id;
#endif
                mn2 = __builtin_amdgcn_fmed3f(mn1, m, mn2);
                mn1 = fminf(mn1, m);
                tot ^= __float_as_uint(x);
            });
            if constexpr (early) unsat |= __ballot((int)par < 0);
            tot &= 0x80000000u;
            const float M1 = mag_of<NORM>(mn1, alpha, beta, clamp);
            const float M2 = mag_of<NORM>(mn2, alpha, beta, clamp);
            uint32_t sg = 0;
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int j = C::COL[r][t], s = C::SH[r][t];
#if QC_ID_AT_VN
                // the min slot is the one with |v| == min1; if several tie, min2 == min1 and M2 == M1,
                // so the choice (and the stored argmin) cannot change any value: bit-exact vs the oracle
                const bool ismin = fabsf(v[t]) == mn1;
                const float mg = ismin ? M2 : M1;
                id = ismin ? (uint32_t)t : id;
#else
                const float mg = (id == (uint32_t)t) ? M2 : M1;
#endif
                const float c = __uint_as_float(__float_as_uint(mg) | ((tot ^ __float_as_uint(v[t])) & 0x80000000u));
                sg = __builtin_amdgcn_alignbit(sg, __float_as_uint(c), 31);
                float cr;
                if constexpr (s == 0) {
                    cr = c;
                } else {
#if QC_ADDR_SGPR_MASK
                    const int addr = sel_lanes<lane_range_mask<Z, CPW>(s, Z)>(br, bmr) + 4 * (Z - s);
#else
                    const int addr = ((zr >= s) ? bmr : br) + 4 * (Z - s);
#endif
                    cr = bperm(addr, c);
                }
                nap[j] = nap[j] + cr;
            });
            mag1[r] = M1;
            mag2[r] = M2;
            pk[r] = sg | (id << 27);
        });
        if constexpr (early) {
            // APP_{it} (this iteration's input) satisfied every check of this codeword: freeze it; the
            // lanes keep running for the wave's other codeword, and their nap is discarded.
            const bool conv = (it > 0) && ((unsat & grp) == 0);
            if (conv && !done) used = it;
            done = done || conv;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const float nx = QUANT ? fminf(fmaxf(nap[j], -app_max), app_max) : nap[j];
                app[j] = done ? app[j] : nx;
            }
            running = !__all(done);
        } else {
#pragma unroll
            for (int j = 0; j < NB; ++j) app[j] = QUANT ? fminf(fmaxf(nap[j], -app_max), app_max) : nap[j];
        }
    }
    if (valid) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const float zz = 0.5f * app[j];
            if (bits) bits[cw * N + j * Z + z] = (uint8_t)(zz <= kZthrF32);
            if (soft) soft[cw * N + j * Z + z] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + expf(-zz));
        }
    }
    if (valid && z == 0 && iters_used) iters_used[cw] = used;
}

template <class C>
static int launch_ms(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft, int32_t* used,
                     hipStream_t st) {
    constexpr int CPW = (C::Z <= 32) ? 2 : 1;
    const int64_t waves = (B + CPW - 1) / CPW;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    const bool es = (p.flags & LDPC_F_EARLY_STOP) != 0;
    const float* x = (const float*)llr;
    float* sf = (float*)soft;
    if (p.algo == LDPC_ALGO_QMIN_SUM) {
        const float qm = (float)p.qmax, am = (float)p.app_max, b = (float)(int)p.beta, qi = 1.0f / p.qstep;
#define QL(E, N) k_qc_ms<C, true, E, N><<<blocks, 256, 0, st>>>(x, B, p.iters, qm, 1.0f, b, qm, am, qi, p.flags, bits, sf, used)
        if (b != 0.0f) { if (es) QL(true, NORM_BETA); else QL(false, NORM_BETA); }
        else           { if (es) QL(true, NORM_PLAIN); else QL(false, NORM_PLAIN); }
#undef QL
    } else {
        const int norm = (p.alpha != 1.0f ? NORM_ALPHA : 0) | (p.beta != 0.0f ? NORM_BETA : 0);
#define FL(E, N) k_qc_ms<C, false, E, N><<<blocks, 256, 0, st>>>(x, B, p.iters, p.clamp, p.alpha, p.beta, 0.f, 0.f, 1.f, p.flags, bits, sf, used)
#define FL2(N) do { if (es) FL(true, N); else FL(false, N); } while (0)
        switch (norm) {
            case NORM_PLAIN: FL2(NORM_PLAIN); break;
            case NORM_ALPHA: FL2(NORM_ALPHA); break;
            case NORM_BETA: FL2(NORM_BETA); break;
            default: FL2(NORM_BOTH);
        }
#undef FL2
#undef FL
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "qc kernel launch: %s", hipGetErrorString(e));
    return LDPC_OK;
}

#define SPEC(C) {C::MB, C::NB, C::Z, &C::COL[0][0], &C::SH[0][0], &C::DEG[0], C::MAXDC, C::NAME, &launch_ms<C>}
static const QCSpec kSpecs[] = {SPEC(Wifi648_12), SPEC(Wifi1296_23)};
#undef SPEC

const QCSpec* qc_lookup(int mb, int nb, int z, const int32_t* shifts) {
    for (const QCSpec& s : kSpecs) {
        if (s.mb != mb || s.nb != nb || s.z != z) continue;
        bool eq = true;
        for (int r = 0; r < mb && eq; ++r) {
            int t = 0;
            for (int j = 0; j < nb; ++j) {
                const int want = (t < s.deg[r] && s.col[r * s.maxdc + t] == j) ? s.sh[r * s.maxdc + t] : -1;
                if (want >= 0) ++t;
                if (shifts[(size_t)r * nb + j] != want) { eq = false; break; }
            }
        }
        if (eq) return &s;
    }
    return nullptr;
}

int qc_z(const QCSpec* s) { return s ? s->z : 0; }

bool qc_supports(const QCSpec* s, const ldpc_params& p) {
    if (!s) return false;
    if (p.flags & LDPC_F_F64) return false;
    return p.algo == LDPC_ALGO_MIN_SUM || p.algo == LDPC_ALGO_QMIN_SUM;
}

size_t qc_workspace(const QCSpec*, int64_t, const ldpc_params&) { return 0; }

int qc_decode(const QCSpec* s, const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
              int32_t* used, char*, hipStream_t st) {
    return s->launch_ms(llr, B, p, bits, soft, used, st);
}

}  // namespace ldpc
