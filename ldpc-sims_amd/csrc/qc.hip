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
#include "qc_common.h"

#include <cstdint>

namespace ldpc {

#ifndef QC_DIAG_NO_L
#define QC_DIAG_NO_L 0
#endif
#ifndef QC_DIAG_NOCMP
#define QC_DIAG_NOCMP 0
#endif
#ifndef QC_L128
#define QC_L128 1  // lane-major L rows read with ds_read_b128 in the stored min-sum kernel
#endif
#ifndef QC_PIPE
#define QC_PIPE 0  // software-pipelined row order: measured no gain (not latency-bound), kept as an option
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
    const int zb = lane_zb<Z, CPW>(z);
    const int base4 = (half * 32 + zb) * 4;
    const int base4m = base4 - 4 * Z;
    // Lane frames (qc_tables.h PHI): lane z holds variable (j, (z + PHI[j]) mod Z); check labels are
    // rotated too, which is invisible outside.  Circulant (r, j) is then a rotation by SHR[r][t], zero for
    // a spanning tree's worth of circulants.  A pure relabelling: every value is computed exactly as before.
    const int64_t cwbase = valid ? cw * N : 0;  // invalid lanes read element 0 (B >= 1) and discard it
    const float vmask = valid ? 1.0f : 0.0f;
    auto vidx = [&](int zz, int j, int phi) {  // index of this lane's variable of block column j
        int t = zz + phi;
        t -= (t >= Z) ? Z : 0;
        return cwbase + j * Z + (valid ? t : 0);
    };
    constexpr bool early = EARLY;

    // channel LLRs L = -llr (quantized in QUANT mode) staged once in LDS: [wave][half][j][z]
    __shared__ float Ls[4 * CPW * N];
    const int lbase = ((threadIdx.x >> 6) * CPW + half) * N + z;
    float app[NB];
    static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        float x = llr[vidx(z, j, C::PHI[j])] * vmask;
        if (QUANT) x = fminf(fmaxf(rintf(x * qinv), -qmax), qmax);
        app[j] = -x;  // L
        if (z < Z) Ls[lbase + j * Z] = app[j];
        app[j] = app[j] + 0.0f;  // APP before iteration 0 = L + sum(c2v = +0): an L of -0 gives +0 (oracle ms_f32_one)
    });
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
        // gather: APP_it of row r's variables rotated into the check frame
        auto gather = [&](auto rr, float* g) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int j = C::COL[r][t], s = C::SHR[r][t];
                if constexpr (s == 0) {
                    g[t] = app[j];
                } else {
                    const int addr = sel_lanes<wrap_mask<Z, CPW>(Z - s)>(base4, base4m) + 4 * s;
                    g[t] = bperm(addr, app[j]);
                }
            });
        };
        // add row r's c2v (already rotated back to the variable frame) into APP_{it+1}, ascending rows
        auto accumulate = [&](auto rr, const float* cr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            // opaque LDS base: else LICM hoists the loop-invariant L reloads out of the loop (+24 VGPRs)
            int lr = lbase;
            asm volatile("" : "+v"(lr));
            static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int j = C::COL[r][t];
                if constexpr (first_row<C>(j) == r) nap[j] = Ls[lr + j * Z];
                nap[j] = nap[j] + cr[t];
            });
        };
        // check-node update of row r from its gathered APPs g: new compressed state, outgoing c2v
        // messages rotated to the variable frame into cr (the rotation is issued, not waited for)
        auto check_row = [&](auto rr, const float* g, float* cr, auto&& between) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            const uint32_t idx_old = pk[r] >> 27;
            float v[d];
            float mn1, mn2;
            uint32_t id = 0, tot = 0;
            uint32_t par = 0;  // bit 31 = parity of the hard decisions of this check's variables
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                const float a = g[t];
                // hard bit(APP) = APP <= thr2 <=> APP - thr2n < 0, thr2n = next float above thr2: a
                // difference of distinct floats is never 0 and never changes sign (denormals kept)
                if constexpr (early) par ^= __float_as_uint(a - thr2n);
                const float om = (idx_old == (uint32_t)t) ? mag2[r] : mag1[r];
                const float old = __uint_as_float(__float_as_uint(om) | ((pk[r] << (31 - (d - 1 - t))) & 0x80000000u));
                float x = a - old;
                if constexpr (QUANT) x = fminf(fmaxf(x, -qmax), qmax);
                v[t] = x;
                tot ^= __float_as_uint(x);
            });
            two_min(v, mn1, mn2);
            if constexpr (early) unsat |= __ballot((int)par < 0);
            between();  // pipelined order: next row's gathers / previous row's adds go here
            tot &= 0x80000000u;
            const float M1 = mag_of<NORM>(mn1, alpha, beta, clamp);
            const float M2 = mag_of<NORM>(mn2, alpha, beta, clamp);
            uint32_t sg = 0;
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int s = C::SHR[r][t];
                // the min slot is the one with |v| == min1; if several tie, min2 == min1 and M2 == M1,
                // so the choice (and the stored argmin) cannot change any value: bit-exact vs the oracle
                const bool ismin = fabsf(v[t]) == mn1;
                const float mg = ismin ? M2 : M1;
                id = ismin ? (uint32_t)t : id;
                const float c = __uint_as_float(__float_as_uint(mg) | ((tot ^ __float_as_uint(v[t])) & 0x80000000u));
                sg = __builtin_amdgcn_alignbit(sg, __float_as_uint(c), 31);
                if constexpr (s == 0) {
                    cr[t] = c;
                } else {
                    const int addr = sel_lanes<wrap_mask<Z, CPW>(s)>(base4, base4m) + 4 * (Z - s);
                    cr[t] = bperm(addr, c);
                }
            });
            asm("" : "+v"(id));  // keep the argmin a small integer (else the shift folds into per-slot constants)
            mag1[r] = M1;
            mag2[r] = M2;
            pk[r] = sg | (id << 27);
        };
#if QC_PIPE
        // software-pipelined rows: row r+1's gathers are issued and row r-1's rotated c2v are added while
        // row r computes, so no row waits on its own LDS round trips.  Per column the adds stay in
        // ascending row order: bit-exact.
        float gA[C::MAXDC], gB[C::MAXDC], cA[C::MAXDC], cB[C::MAXDC];
        gather(std::integral_constant<int, 0>{}, gA);
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            float* gcur = (r & 1) ? gB : gA;
            float* gnxt = (r & 1) ? gA : gB;
            float* ccur = (r & 1) ? cB : cA;
            float* cprv = (r & 1) ? cA : cB;
            check_row(rr, gcur, ccur, [&]() __attribute__((always_inline)) {
                if constexpr (r + 1 < MB) gather(std::integral_constant<int, r + 1>{}, gnxt);
                if constexpr (r >= 1) accumulate(std::integral_constant<int, r - 1>{}, cprv);
            });
        });
        accumulate(std::integral_constant<int, MB - 1>{}, ((MB - 1) & 1) ? cB : cA);
#else
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            float g[C::MAXDC], c[C::MAXDC];
            gather(rr, g);
            check_row(rr, g, c, []() {});
            accumulate(rr, c);
        });
#endif
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
        int zo = z;  // opaque: the store indices must not be CSE'd with the load indices (48 VGPRs live)
        asm volatile("" : "+v"(zo));
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            const int64_t o = vidx(zo, j, C::PHI[j]);
            const float zz = 0.5f * app[j];
            if (bits) bits[o] = (uint8_t)(zz <= kZthrF32);
            if (soft) soft[o] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + expf(-zz));
        });
    }
    if (valid && z == 0 && iters_used) iters_used[cw] = used;
}

// Stored-message variant (fixed iteration count): every edge's c2v message is kept in a VGPR in the
// VARIABLE frame, so the check update needs no reconstruction from a compressed state and the variable
// update no re-compression.  Per iteration: v2c = APP - c2v in place for all edges (APP is then dead),
// then per row: gather v2c into the check frame, two-minimum + sign product, scatter the new c2v back
// (in place) and add it into APP_{it+1} in ascending row order.  Same arithmetic as k_qc_ms / the
// oracle, operation for operation.  The register kernel is instruction-fetch bound (SQC_ICACHE_BUSY ~
// 100%): this form executes ~12 instead of ~17 instructions (~76 instead of ~124 bytes) per edge, at
// <= 128 VGPRs (4 waves per SIMD).
// LDS-row rotations in the stored min-sum / tanh-SP kernels: off — neither is LDS-pipe bound; A/B slower in
// every configuration ((1296,2/3) min-sum 42.1 -> 38.6, early stop 52.3 -> 44.0; (648,1/2) tanh-SP 6.75 ->
// 6.64, early stop 12.35 -> 11.83; (1296,2/3) tanh-SP 3.32 -> 3.28 M cw/s)
#ifndef QC_ST_LDSROT
#define QC_ST_LDSROT 0
#endif
#ifndef QC_ST_LDSROT_EARLY
#define QC_ST_LDSROT_EARLY 0
#endif
#ifndef QC_SP_LDSROT
#define QC_SP_LDSROT 0
#endif
#ifndef QC_SP_LDSROT_EARLY
#define QC_SP_LDSROT_EARLY 0
#endif
#ifndef QC_ST_TPB
#define QC_ST_TPB 256  // threads per workgroup of the stored min-sum kernel (whole waves)
#endif
// Early stop: a workgroup's LDS stays allocated until its slowest wave exits, so with waves that leave at
// different iterations one-wave workgroups free CU slots sooner (A/B, profiles/r02/ab/ab_tpb.txt: (648,1/2)
// min-sum early stop 61.9 -> 65.5 M cw/s; fixed-count kernels: 256 / 128 / 64 within noise, 256 kept).
#ifndef QC_ST_TPB_EARLY
#define QC_ST_TPB_EARLY 64
#endif
#ifndef QC_SP_TPB_EARLY
#define QC_SP_TPB_EARLY 64  // tanh-SP early stop (k_qc_sp_st): 12.35 -> 13.97 M cw/s
#endif
template <bool EARLY>
constexpr int st_tpb() { return EARLY ? QC_ST_TPB_EARLY : QC_ST_TPB; }
template <bool EARLY>
constexpr int sp_tpb() { return EARLY ? QC_SP_TPB_EARLY : 256; }
#ifndef QC_ST_WAVES_PER_SIMD
#define QC_ST_WAVES_PER_SIMD 3  // dispatched for Z > 32 ((1296,2/3)): spill-free at 134 VGPRs, 41.0 vs 39.9 M cw/s at 4
                                // waves (2-5 VGPRs spilled; A/B, 20 it)
#endif
#ifndef QC_ST_ES_ROWS
#define QC_ST_ES_ROWS 1  // early stop, one codeword per wave: syndrome row by row with an early exit; A/B (1296,2/3)
                         // 20 it (profiles/r03/ab/ab_st_esrows.txt): 54.4-54.9 -> 58.5-59.0 M cw/s in qc_es.hip
#endif
#ifndef QC_ST_WAVES_PER_SIMD_EARLY
#define QC_ST_WAVES_PER_SIMD_EARLY 4  // early stop keeps APP_it and the syndrome ballots live: 14-15 VGPRs spill at
                                      // 4 waves, yet 3 waves (spill-free) measured 9 % slower on (1296,2/3)
#endif

template <class C, bool QUANT, bool EARLY, int NORM>
__global__ __launch_bounds__(256, EARLY ? QC_ST_WAVES_PER_SIMD_EARLY : QC_ST_WAVES_PER_SIMD) void k_qc_ms_st(const float* __restrict__ llr, int64_t B, int iters,
                                                                       float clamp, float alpha, float beta, float qmax,
                                                                       float app_max, float qinv, int flags,
                                                                       uint8_t* __restrict__ bits, float* __restrict__ soft,
                                                                       int32_t* __restrict__ iters_used) {
    constexpr int Z = C::Z, NB = C::NB, MB = C::MB, N = NB * Z;
    constexpr int NE = edge_off<C>(MB);
    static_assert(Z <= 64, "register kernel needs Z <= 64");
    constexpr int CPW = (Z <= 32) ? 2 : 1;
    const int lane = threadIdx.x & 63;
    const int half = (CPW == 2) ? (lane >> 5) : 0;
    const int z = (CPW == 2) ? (lane & 31) : lane;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t cw = wave * CPW + half;
    const bool valid = (z < Z) && (cw < B);
    const int zb = lane_zb<Z, CPW>(z);
    const int base4 = (half * 32 + zb) * 4;
    const int base4m = base4 - 4 * Z;
    // lane rotations through a per-wave LDS row instead of ds_bpermute (see QC_PH_LDSROT)
    constexpr bool LDSROT = EARLY ? QC_ST_LDSROT_EARLY : QC_ST_LDSROT;
    __shared__ float Rw[LDSROT ? 256 : 1];
    const int wrow = LDSROT ? (int)(threadIdx.x & ~63u) * 4 : 0;
    if constexpr (LDSROT) {
        const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(&Rw[0]) + (unsigned)wrow);
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" ::"s"(m0) : "memory");
    }
    auto xfer = [&](int addr, float x) __attribute__((always_inline)) {
        if constexpr (LDSROT) {
            asm volatile("ds_write_addtid_b32 %0" ::"v"(x) : "memory");
            return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(Rw) + wrow + addr);
        } else {
            return bperm(addr, x);
        }
    };
    const int64_t cwbase = valid ? cw * N : 0;
    const float vmask = valid ? 1.0f : 0.0f;
    auto vidx = [&](int zz, int j, int phi) {
        int t = zz + phi;
        t -= (t >= Z) ? Z : 0;
        return cwbase + j * Z + (valid ? t : 0);
    };
#if QC_L128
    using f4 = __attribute__((ext_vector_type(4))) float;
    constexpr int LSTR = lstr<C>(), NG = (NB + 3) / 4;
    __shared__ __attribute__((aligned(16))) float Ls[st_tpb<EARLY>() * LSTR];  // lane-major L rows (qc_common.h lpos)
    const int lrow = threadIdx.x * LSTR;
#define LS_AT(row, j) Ls[(row) + lpos<C>(j)]
#else
    __shared__ float Ls[(st_tpb<EARLY>() / 64) * CPW * N];
    const int lrow = ((threadIdx.x >> 6) * CPW + half) * N + z;
#define LS_AT(row, j) Ls[(row) + (j) * Z]
#endif
    float app[NB];
    static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        float x = llr[vidx(z, j, C::PHI[j])] * vmask;
        if (QUANT) x = fminf(fmaxf(rintf(x * qinv), -qmax), qmax);
        app[j] = -x;  // L
        if (QC_L128 || z < Z) LS_AT(lrow, j) = app[j];
        app[j] = app[j] + 0.0f;  // APP_0 = L + sum(c2v = +0): -0 -> +0, as the oracle
    });
    if (QUANT) {
#pragma unroll
        for (int j = 0; j < NB; ++j) app[j] = fminf(fmaxf(app[j], -app_max), app_max);
    }
    float msg[NE];  // c2v of every edge (variable frame); v2c in place during an iteration
#pragma unroll
    for (int e = 0; e < NE; ++e) msg[e] = 0.0f;
    // early stop: lanes of each codeword group, converged groups, their iteration counts
    constexpr uint64_t ACTIVE = lane_range_mask<Z, CPW>(0, Z);
    uint64_t done_groups = 0;  // (group lane mask) of converged codewords, CPW == 2
    int used_lo = iters, used_hi = iters;

    for (int it = 0; it < iters; ++it) {
        if constexpr (EARLY) {
            if (it > 0) {
                // syndrome of APP_it: per block column one ballot of the hard decisions (bit = APP <= 2*ZTHR;
                // quantized: APP < 0, the same for integers), then per check row the XOR of its columns'
                // masks rotated into the check frame by the edge's lane shift
                const float thr2 = 2.0f * kZthrF32;
                if constexpr (QC_ST_ES_ROWS && CPW == 1) {
                    // row by row with an early exit (as k_qc_ms_ph's QC_PH_ES_ROWS): the codeword is still
                    // unsatisfied once one row's parity is nonzero, usually at the first row
                    bool sat = true;
                    static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                        constexpr int r = decltype(rr)::value;
                        if (sat) {
                            uint64_t par = 0;
                            static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                                constexpr int t = decltype(tt)::value;
                                const uint64_t b = __ballot(app[C::COL[r][t]] <= thr2) & ACTIVE;
                                par ^= rot_lanes<Z, CPW, C::SHR[r][t]>(b);
                            });
                            if (par & ACTIVE) sat = false;
                        }
                    });
                    if (sat) {  // the wave's codeword satisfies every check: APP_it is the output
                        used_lo = it;
                        break;
                    }
                } else {
                uint64_t par[MB];
#pragma unroll
                for (int r = 0; r < MB; ++r) par[r] = 0;
                static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                    constexpr int j = decltype(jj)::value;
                    const uint64_t b = __ballot(app[j] <= thr2) & ACTIVE;
                    static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                        constexpr int r = decltype(rr)::value;
                        constexpr int t = first_slot<C>(r, j);
                        if constexpr (t >= 0) par[r] ^= rot_lanes<Z, CPW, C::SHR[r][t]>(b);
                    });
                });
                uint64_t unsat = 0;
#pragma unroll
                for (int r = 0; r < MB; ++r) unsat |= par[r];
                unsat &= ACTIVE;
                if constexpr (CPW == 1) {
                    if (unsat == 0) {  // the wave's codeword satisfies every check: APP_it is the output
                        used_lo = it;
                        break;
                    }
                } else {
                    constexpr uint64_t G0 = lane_range_mask<Z, 1>(0, Z), G1 = G0 << 32;
                    const uint64_t newly = ((unsat & G0) ? 0 : G0) | ((unsat & G1) ? 0 : G1);
                    const uint64_t fresh = newly & ~done_groups;
                    if (fresh) {
                        // park the converged codeword's APP_it in its own L region of LDS (L is no longer
                        // needed by it); its lanes keep computing for the other codeword, discarded
                        if (fresh & G0) used_lo = it;
                        if (fresh & G1) used_hi = it;
                        if ((fresh >> lane) & 1ull) {
                            static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                                constexpr int j = decltype(jj)::value;
                                LS_AT(lrow, j) = app[j];
                            });
                        }
                        done_groups |= fresh;
                        if (done_groups == (G0 | G1)) break;
                    }
                }
                }  // all rows
            }
        }
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int e = edge_off<C>(r) + t;
                float x = app[C::COL[r][t]] - msg[e];
                if constexpr (QUANT) x = fminf(fmaxf(x, -qmax), qmax);
                msg[e] = x;
            });
        });
        float nap[NB];
#if QC_L128
        f4 Lg[NG];
#endif
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            constexpr int e0 = edge_off<C>(r);
#if QC_L128
            static_for<0, NG>([&](auto gg) __attribute__((always_inline)) {
                constexpr int g = decltype(gg)::value;
                if constexpr (lgroup_row<C>(g) == r) {
                    int lr = lrow;
                    asm volatile("" : "+v"(lr));  // not hoisted out of the iteration (register budget)
                    Lg[g] = *static_cast<const f4*>(__builtin_assume_aligned(&Ls[lr + 4 * g], 16));
                }
            });
#endif
            float v[d];
            float mn1, mn2;
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int s = C::SHR[r][t];
                float x;
                if constexpr (s == 0) {
                    x = msg[e0 + t];
                } else {
                    const int addr = sel_lanes<wrap_mask<Z, CPW>(Z - s)>(base4, base4m) + 4 * s;
                    x = xfer(addr, msg[e0 + t]);
                }
                v[t] = x;
            });
            two_min(v, mn1, mn2);
            const uint32_t tot = xor_all(v) & 0x80000000u;
            // sign of the product folded into the two magnitudes once per row
            const float M1 = __uint_as_float(__float_as_uint(mag_of<NORM>(mn1, alpha, beta, clamp)) ^ tot);
            const float M2 = __uint_as_float(__float_as_uint(mag_of<NORM>(mn2, alpha, beta, clamp)) ^ tot);
            // NORM_PLAIN: compare-free select (med3 of the unsigned magnitudes, XOR): +3.4 % on (1296,2/3), A/B;
            // -1.3 % in the LDS-bound k_qc_ms_ph, which keeps v_cmp/v_cndmask
            const float A1 = mag_of<NORM>(mn1, alpha, beta, clamp), A2 = mag_of<NORM>(mn2, alpha, beta, clamp);
            const uint32_t X = __float_as_uint(M1) ^ __float_as_uint(A2);
#if !QC_L128
            int lr = lrow;
            asm volatile("" : "+v"(lr));
#endif
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int j = C::COL[r][t], s = C::SHR[r][t];
                // |v| == min1 picks the min slot; ties imply min2 == min1 (bit-exact, see k_qc_ms)
#if QC_DIAG_NOCMP
                const float mg = M1;  // DIAGNOSTIC BUILD ONLY (wrong results): prices the argmin select
                const float c = __uint_as_float(__float_as_uint(mg) ^ (__float_as_uint(v[t]) & 0x80000000u));
#else
                float c;
                if constexpr (NORM == NORM_PLAIN) {
                    const uint32_t m = __float_as_uint(__builtin_amdgcn_fmed3f(fabsf(v[t]), A1, A2));
                    c = __uint_as_float((X ^ m) ^ (__float_as_uint(v[t]) & 0x80000000u));
                } else {
                    const float mg = (fabsf(v[t]) == mn1) ? M2 : M1;
                    c = __uint_as_float(__float_as_uint(mg) ^ (__float_as_uint(v[t]) & 0x80000000u));
                }
#endif
                float cr;
                if constexpr (s == 0) {
                    cr = c;
                } else {
                    const int addr = sel_lanes<wrap_mask<Z, CPW>(s)>(base4, base4m) + 4 * (Z - s);
                    cr = xfer(addr, c);
                }
                msg[e0 + t] = cr;
#if QC_DIAG_NO_L
                // DIAGNOSTIC BUILD ONLY (wrong results): no per-iteration L reads, to price them
                if constexpr (first_row<C>(j) == r) nap[j] = 0.0f;
#elif QC_L128
                if constexpr (first_row<C>(j) == r) nap[j] = Lg[lpos<C>(j) / 4][lpos<C>(j) % 4];
#else
                if constexpr (first_row<C>(j) == r) nap[j] = Ls[lr + j * Z];
#endif
                nap[j] = nap[j] + cr;
            });
        });
#pragma unroll
        for (int j = 0; j < NB; ++j) app[j] = QUANT ? fminf(fmaxf(nap[j], -app_max), app_max) : nap[j];
    }
    // epilogue indices recomputed from the thread id (opaque), so nothing but the loop state is live
    // across the loop (the 4-waves/SIMD register budget is 128)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int zo = (CPW == 2) ? (tid & 31) : (tid & 63);
    const int64_t cwo = (((int64_t)blockIdx.x * blockDim.x + tid) >> 6) * CPW + ((CPW == 2) ? ((tid >> 5) & 1) : 0);
    const bool parked = EARLY && CPW == 2 && ((done_groups >> (tid & 63)) & 1ull);
    if (zo < Z && cwo < B) {
#if QC_L128
        const int lbo = tid * LSTR;
#else
        const int lbo = ((tid >> 6) * CPW + ((CPW == 2) ? ((tid >> 5) & 1) : 0)) * N + zo;
#endif
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            int t = zo + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            const int64_t o = cwo * N + j * Z + t;
            const float zz = 0.5f * (parked ? LS_AT(lbo, j) : app[j]);
            if (bits) bits[o] = (uint8_t)(zz <= kZthrF32);
            if (soft) soft[o] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + expf(-zz));
        });
        if (zo == 0 && iters_used) iters_used[cwo] = (CPW == 2 && ((tid >> 5) & 1)) ? used_hi : used_lo;
    }
}
#undef LS_AT

// ---- Phased stored-message min-sum (k_qc_ms_ph) ---------------------------------------------------
// The same flooding arithmetic as k_qc_ms_st (and the oracle), operation for operation, regrouped into
// two phases per iteration so that no lane rotation sits on a dependency chain:
//   CN phase, row by row:   msg[e] (v2c, variable frame) -> gathered into the check frame IN PLACE,
//                           two-minimum / sign product, msg[e] = new c2v in the CHECK frame.
//                           Rows are independent: row r+1's gathers overlap row r's arithmetic.
//   VN phase, column by column: msg[e] -> rotated back to the variable frame in place,
//                           APP_j = L_j + sum of c2v in ascending row order (the oracle's order),
//                           msg[e] = APP_j - c2v (v2c of the next iteration).  Columns are independent.
// Nothing but msg[] is live across a phase (APP is per column and transient), so the rotation
// addresses — one per distinct lane shift rho, "read lane (z + rho) mod Z of my group" — are computed
// once before the loop and held in registers (QC_PH_ADDR_MIN_USES) instead of one v_cndmask per ds_bpermute.
// Iteration 0's v2c is L itself (c2v = +0: L - 0 == L bitwise, also for L = -0), so the loop starts at
// the CN phase; the last iteration's VN phase writes the outputs directly instead of forming v2c.
#ifndef QC_PH_ADDR_MIN_USES
#define QC_PH_ADDR_MIN_USES 3  // rotations used >= 3 times per iteration get an address register (A/B: 1 -> spills, 38.5 vs 37.9 M cw/s at 1; 4: 38.3; 6: 37.7; none: 37.0)
#endif
#ifndef QC_PH_WAVES_PER_SIMD
#define QC_PH_WAVES_PER_SIMD 4
#endif
#ifndef QC_PH_ADDR_MIN_USES_EARLY
#define QC_PH_ADDR_MIN_USES_EARLY QC_PH_ADDR_MIN_USES
#endif
// Phase priorities (s_setprio, round 4): a SIMD issues from the higher-priority waves first, so raising the phase
// whose waves stall on their own dependences lets their instructions issue the moment they are ready while the
// other phase's independent work fills the gaps.  A/B profiles/r04/ab/ab_prio.txt.
#ifndef QC_PH_PRIO
// phased min-sum, fixed count: 2 = s_setprio 1 over the CN phase (the rotations' gathers and the two-minimum
// chains), 0 over the VN phase: 42.0 -> 43.4-44.0 M cw/s; 1 = the reverse (-0.7 %); 3 = 2 with the VN phase's
// first lookahead rotations still at 1
#define QC_PH_PRIO 2
#endif
#ifndef QC_SP_PRIO
// tanh-SP register kernel, fixed count: 2 = s_setprio 1 over the VN phase (exp chains), 0 over the rows: 16.2 ->
// 16.6 M cw/s; 1 = priority over each row's gather only (neutral)
#define QC_SP_PRIO 2
#endif
#ifndef QC_PH_LA
#define QC_PH_LA 1  // rotations issued this many rows / columns ahead, in place: +2.5 % (A/B 38.9 vs 38.0 M cw/s; 2: +2.0 %, 3: +1.5 %; 0: the plain phased order)
#endif
// QC_PH_LDSROT: lane rotations through a 256-B LDS row per wave instead of ds_bpermute — every lane stores its
// value with ds_write_addtid_b32 (address M0 + 4 * lane: no address VGPR to move), then loads the slot of lane
// (z + rho) with ds_read_b32 at the address the ds_bpermute would have taken.  A wave's LDS operations run in
// order, so one row serves every rotation with no wait or barrier.  Measured on the box
// (scripts/lds_micro.hip, profiles/r02/micro/): 4.31 LDS-pipe cycles per rotation against 6.16 for ds_bpermute
// (which moves an address and a data VGPR in and a data VGPR out) — the resource that binds this kernel.
#ifndef QC_PH_LDSROT
#define QC_PH_LDSROT 1
#endif
#ifndef QC_SP_MASK_IDLE
#define QC_SP_MASK_IDLE 0  // A/B neutral (+0.2 %, profiles/r04/ab/ab_mask.txt)
#endif
#ifndef QC_PH_MASK_IDLE
#define QC_PH_MASK_IDLE 1  // A/B profiles/r04/ab/ab_mask.txt: +0.9 % (42.02 -> 42.39 M cw/s, three interleaved pairs), parity green
#endif
#ifndef QC_PH_XSEL
#define QC_PH_XSEL 0  // compare-free check output in the lookahead loop (plain min-sum): A/B with LDS-row
                      // rotations 43.05 vs 43.13 M cw/s (removes the 60 hazard s_nops, same VALU count) — off
#endif
#ifndef QC_PH_LDSROT_EARLY
#define QC_PH_LDSROT_EARLY 0  // early stop keeps ds_bpermute (A/B: 61.8 vs 61.5 M cw/s; not LDS-bound)
#endif
// QC_PH_APPB (fixed iteration count, LDS-row rotations): v2c is formed in the CHECK frame.  The VN phase
// rotates each c2v back into a temporary for the APP sum (c2v itself stays in the check frame), stores APP_j
// into the wave's row ONCE and every edge of column j reads it at its own shift: v2c = rot_s(APP_j) - c2v,
// the same subtraction of the same two values as APP_j - c2v followed by the gather.  The CN phase then needs
// no rotation; per iteration 44 + 18 row stores instead of 88 on (648,1/2), the same 88 reads.
#ifndef QC_PH_APPB
#define QC_PH_APPB 0  // A/B -5 % (no lookahead) / -3.5 % (lookahead, spills): profiles/r02/ab/ab_appb.txt
#endif
#ifndef QC_PH_APPB_LA
#define QC_PH_APPB_LA 1  // back-rotations of column p + 1 issued before column p's sum (0: in the column's own order)
#endif
#ifndef QC_PH_ES_ROWS
#define QC_PH_ES_ROWS 1  // early stop: syndrome row by row with an early exit.  A/B (648,1/2) 50 it
#endif                   // (profiles/r03/ab/ab_ph_esrows.txt): SQ_INSTS_SALU 495 M per launch against 864 M VALU in
                         // the all-rows form; the row scan built with the default scheduler (qc_es.hip, 13
                         // VGPRs spilled) 62.9-66.4 -> 69.7-70.3 M cw/s; under iterative-ILP it spills 63 (with 5
                         // address registers spill-free: 67.5-68.0)
#ifndef QC_PH_WAVES_PER_SIMD_EARLY
#define QC_PH_WAVES_PER_SIMD_EARLY 3  // spill-free (145 VGPRs): 648 min-sum early stop 24.6 -> 57.9 M cw/s (A/B)
#endif

template <class C, bool QUANT, bool EARLY, int NORM>
__global__ __launch_bounds__(256, EARLY ? QC_PH_WAVES_PER_SIMD_EARLY : QC_PH_WAVES_PER_SIMD) void k_qc_ms_ph(const float* __restrict__ llr, int64_t B, int iters,
                                                                       float clamp, float alpha, float beta, float qmax,
                                                                       float app_max, float qinv, int flags,
                                                                       uint8_t* __restrict__ bits, float* __restrict__ soft,
                                                                       int32_t* __restrict__ iters_used) {
    constexpr int Z = C::Z, NB = C::NB, MB = C::MB, N = NB * Z;
    constexpr int NE = edge_off<C>(MB);
    static_assert(Z <= 32, "phased kernel: two codewords per wave (Z <= 32)");
    constexpr int CPW = 2;
    const int lane = threadIdx.x & 63;
    const int half = lane >> 5;
    const int z = lane & 31;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t cw = wave * CPW + half;
    const bool valid = (z < Z) && (cw < B);
    const int zb = lane_zb<Z, CPW>(z);
    const int base4 = (half * 32 + zb) * 4;
    const int base4m = base4 - 4 * Z;
    using f4 = __attribute__((ext_vector_type(4))) float;
    constexpr int LSTR = lstr<C>();
    __shared__ __attribute__((aligned(16))) float Ls[st_tpb<EARLY>() * LSTR];  // lane-major L rows (qc_common.h lpos)
    const int lrow = threadIdx.x * LSTR;
    const int lrow4 = lrow * 4;  // bytes (lds_reload)

    constexpr bool LDSROT = EARLY ? QC_PH_LDSROT_EARLY : QC_PH_LDSROT;
    __shared__ float Rw[LDSROT ? st_tpb<EARLY>() : 1];  // one 64-lane rotation row per wave
    const int wrow = LDSROT ? (int)(threadIdx.x & ~63u) * 4 : 0;  // this wave's row, bytes from Rw
    const int rb4 = base4 + wrow, rb4m = base4m + wrow;        // read addresses include the row
    if constexpr (LDSROT) {
        // M0 = this wave's row, set once: nothing else in this kernel reads or writes M0 (the CPU test
        // test_kernel_resources.py::test_headline_m0_written_once checks the built code); s_nop 0: an SALU write
        // of M0 needs one wait state before an add-TID LDS instruction reads it
        const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(&Rw[0]) + (unsigned)wrow);
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" ::"s"(m0) : "memory");
    }
    auto xfer = [&](int addr, float x) __attribute__((always_inline)) {
        if constexpr (LDSROT) {
            asm volatile("ds_write_addtid_b32 %0" ::"v"(x) : "memory");
            return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(Rw) + addr);
        } else {
            return bperm(addr, x);
        }
    };
    // rotation addresses, one register per distinct shift used often enough (the others: one v_cndmask
    // per use, as k_qc_ms_st)
    constexpr int AMU = EARLY ? QC_PH_ADDR_MIN_USES_EARLY : QC_PH_ADDR_MIN_USES;
    int ra[Z];
    static_for<1, Z>([&](auto rr) __attribute__((always_inline)) {
        constexpr int rho = decltype(rr)::value;
        if constexpr (rot_uses<C>(rho) >= AMU)
            ra[rho] = sel_lanes<wrap_mask<Z, CPW>(Z - rho)>(rb4, rb4m) + 4 * rho;
    });
    auto rot = [&](auto rr, float x) __attribute__((always_inline)) {  // value of lane (z + rho) mod Z
        constexpr int rho = decltype(rr)::value;
        if constexpr (rho == 0) {
            return x;
        } else if constexpr (rot_uses<C>(rho) >= AMU) {
            return xfer(ra[rho], x);
        } else {
            return xfer(sel_lanes<wrap_mask<Z, CPW>(Z - rho)>(rb4, rb4m) + 4 * rho, x);
        }
    };
    (void)ra;

    // L = -llr (quantized in QUANT mode) into this lane's LDS row; msg = v2c of iteration 0 = APP_0 = L
    float msg[NE];
    {
        const int64_t cwbase = valid ? cw * N : 0;
        const float vmask = valid ? 1.0f : 0.0f;
        float L[NB];
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            int t = z + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            float x = llr[cwbase + j * Z + (valid ? t : 0)] * vmask;
            if (QUANT) x = fminf(fmaxf(rintf(x * qinv), -qmax), qmax);
            L[j] = -x;
            Ls[lrow + lpos<C>(j)] = L[j];
            if (QUANT) L[j] = fminf(fmaxf(L[j], -app_max), app_max);  // APP_0 (k_qc_ms_st: app clamp)
        });
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                float x = L[C::COL[r][t]] + 0.0f;  // v2c = APP_0 - c2v(= +0), APP_0 = L + (+0): -0 -> +0
                if constexpr (QUANT) x = fminf(fmaxf(x, -qmax), qmax);
                msg[edge_off<C>(r) + t] = x;
            });
        });
    }
    constexpr uint64_t ACTIVE = lane_range_mask<Z, CPW>(0, Z);
    constexpr uint64_t G0 = lane_range_mask<Z, 1>(0, Z), G1 = G0 << 32;
    uint64_t done_groups = 0;
    int used_lo = iters, used_hi = iters;
    const float thr2 = 2.0f * kZthrF32;

    // CN phase: v2c (variable frame) -> c2v (check frame), in place
    auto cn_phase = [&]() __attribute__((always_inline)) {
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            constexpr int e0 = edge_off<C>(r);
            float v[d];
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                v[t] = rot(std::integral_constant<int, C::SHR[r][t]>{}, msg[e0 + t]);
            });
            float mn1, mn2;
            two_min(v, mn1, mn2);
            const uint32_t tot = xor_all(v) & 0x80000000u;
            const float M1 = __uint_as_float(__float_as_uint(mag_of<NORM>(mn1, alpha, beta, clamp)) ^ tot);
            const float M2 = __uint_as_float(__float_as_uint(mag_of<NORM>(mn2, alpha, beta, clamp)) ^ tot);
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                const float mg = (fabsf(v[t]) == mn1) ? M2 : M1;
                msg[e0 + t] = __uint_as_float(__float_as_uint(mg) ^ (__float_as_uint(v[t]) & 0x80000000u));
            });
        });
    };
#if QC_PH_LA
    // Lookahead form (A/B): rotations happen in place on msg[] (no extra registers), issued QC_PH_LA rows /
    // columns ahead of the arithmetic that consumes them, so each wave keeps several ds_bpermute in flight
    auto gather_row = [&](auto rr) __attribute__((always_inline)) {
        constexpr int r = decltype(rr)::value;
        static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
            constexpr int t = decltype(tt)::value;
            msg[edge_off<C>(r) + t] = rot(std::integral_constant<int, C::SHR[r][t]>{}, msg[edge_off<C>(r) + t]);
        });
    };
    auto math_row = [&](auto rr) __attribute__((always_inline)) {
        constexpr int r = decltype(rr)::value;
        constexpr int d = C::DEG[r];
        constexpr int e0 = edge_off<C>(r);
        float v[d];
        static_for<0, d>([&](auto tt) __attribute__((always_inline)) { v[decltype(tt)::value] = msg[e0 + decltype(tt)::value]; });
        float mn1, mn2;
        two_min(v, mn1, mn2);
        const uint32_t tot = xor_all(v) & 0x80000000u;
        const float M1 = __uint_as_float(__float_as_uint(mag_of<NORM>(mn1, alpha, beta, clamp)) ^ tot);
        const float M2 = __uint_as_float(__float_as_uint(mag_of<NORM>(mn2, alpha, beta, clamp)) ^ tot);
        if constexpr (QC_PH_XSEL && NORM == NORM_PLAIN) {  // compare-free select, as k_qc_ms_st
            const float A1 = mag_of<NORM>(mn1, alpha, beta, clamp), A2 = mag_of<NORM>(mn2, alpha, beta, clamp);
            const uint32_t X = __float_as_uint(M1) ^ __float_as_uint(A2);
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                const uint32_t m = __float_as_uint(__builtin_amdgcn_fmed3f(fabsf(v[t]), A1, A2));
                msg[e0 + t] = __uint_as_float((X ^ m) ^ (__float_as_uint(v[t]) & 0x80000000u));
            });
        } else {
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                const float mg = (fabsf(v[t]) == mn1) ? M2 : M1;
                msg[e0 + t] = __uint_as_float(__float_as_uint(mg) ^ (__float_as_uint(v[t]) & 0x80000000u));
            });
        }
    };
    auto cn_phase_la = [&]() __attribute__((always_inline)) {
        static_for<0, (QC_PH_LA < MB ? QC_PH_LA : MB)>([&](auto rr) __attribute__((always_inline)) { gather_row(rr); });
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            if constexpr (!EARLY && QC_PH_PRIO == 6) __builtin_amdgcn_s_setprio(1);
            if constexpr (r + QC_PH_LA < MB) gather_row(std::integral_constant<int, r + QC_PH_LA>{});
            if constexpr (!EARLY && QC_PH_PRIO == 6) __builtin_amdgcn_s_setprio(0);
            math_row(rr);
        });
    };
#endif
    // VN phase, column j: c2v back to the variable frame, APP_j = L_j + ascending sum; returns APP_j
    f4 Lg;
    auto vn_col = [&](auto pp) __attribute__((always_inline)) {
        constexpr int p = decltype(pp)::value;  // LDS position (columns in first-use order)
        constexpr int j = lcol<C>(p);
        constexpr int dj = col_deg<C>(j);
        if constexpr (p % 4 == 0) {
            Lg = lds_reload<4 * p, f4, 16>(Ls, lrow4);  // not hoisted out of the loop (register budget)
        }
        float a = Lg[p % 4];
        static_for<0, dj>([&](auto kk) __attribute__((always_inline)) {
            constexpr int e = col_edge<C>(j, decltype(kk)::value);
            constexpr int r = edge_row<C>(e), t = e - edge_off<C>(r);
            constexpr int s = C::SHR[r][t];
            msg[e] = rot(std::integral_constant<int, (s == 0) ? 0 : Z - s>{}, msg[e]);
            a = a + msg[e];
        });
        if (QUANT) a = fminf(fmaxf(a, -app_max), app_max);
        return a;
    };
#if QC_PH_LA
    auto rot_col = [&](auto pp) __attribute__((always_inline)) {  // c2v of column lcol(p) back, in place
        constexpr int j = lcol<C>(decltype(pp)::value);
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) {
            constexpr int e = col_edge<C>(j, decltype(kk)::value);
            constexpr int r = edge_row<C>(e), t = e - edge_off<C>(r);
            constexpr int s = C::SHR[r][t];
            msg[e] = rot(std::integral_constant<int, (s == 0) ? 0 : Z - s>{}, msg[e]);
        });
    };
    auto sum_col = [&](auto pp) __attribute__((always_inline)) {  // APP_j from already rotated c2v
        constexpr int p = decltype(pp)::value;
        constexpr int j = lcol<C>(p);
        if constexpr (p % 4 == 0) {
            Lg = lds_reload<4 * p, f4, 16>(Ls, lrow4);
        }
        float a = Lg[p % 4];
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) { a = a + msg[col_edge<C>(j, decltype(kk)::value)]; });
        if (QUANT) a = fminf(fmaxf(a, -app_max), app_max);
        return a;
    };
#endif
    auto v2c_col = [&](auto jj, float a) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) {
            constexpr int e = col_edge<C>(j, decltype(kk)::value);
            float x = a - msg[e];
            if constexpr (QUANT) x = fminf(fmaxf(x, -qmax), qmax);
            msg[e] = x;
        });
    };

#if QC_PH_LA && QC_PH_APPB
    constexpr bool APPB = !EARLY && LDSROT;
    constexpr int DMX = [] {
        int m = 0;
        for (int j = 0; j < NB; ++j) m = col_deg<C>(j) > m ? col_deg<C>(j) : m;
        return m;
    }();
    auto row_put = [&](float x) __attribute__((always_inline)) {
        asm volatile("ds_write_addtid_b32 %0" ::"v"(x) : "memory");
    };
    auto row_get = [&](auto rr) __attribute__((always_inline)) {  // lane (z + rho) mod Z of the last row_put
        constexpr int rho = decltype(rr)::value;
        int addr;
        if constexpr (rot_uses<C>(rho) >= AMU) addr = ra[rho];
        else addr = sel_lanes<wrap_mask<Z, CPW>(Z - rho)>(rb4, rb4m) + 4 * rho;
        return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(Rw) + addr);
    };
    auto back_col = [&](auto pp, float* T) __attribute__((always_inline)) {  // c2v of column lcol(p), variable frame
        constexpr int j = lcol<C>(decltype(pp)::value);
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) {
            constexpr int e = col_edge<C>(j, decltype(kk)::value);
            constexpr int r = edge_row<C>(e), t = e - edge_off<C>(r);
            constexpr int s = C::SHR[r][t];
            T[decltype(kk)::value] = rot(std::integral_constant<int, (s == 0) ? 0 : Z - s>{}, msg[e]);
        });
    };
    auto bcast_col = [&](auto pp, float a) __attribute__((always_inline)) {  // v2c of column lcol(p), check frames
        constexpr int j = lcol<C>(decltype(pp)::value);
        constexpr bool any = col_deg<C>(j) > 0 && [] {
            for (int k = 0; k < col_deg<C>(j); ++k) {
                const int e = col_edge<C>(j, k), r = edge_row<C>(e);
                if (C::SHR[r][e - edge_off<C>(r)] != 0) return true;
            }
            return false;
        }();
        if constexpr (any) row_put(a);
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) {
            constexpr int e = col_edge<C>(j, decltype(kk)::value);
            constexpr int r = edge_row<C>(e), t = e - edge_off<C>(r);
            constexpr int s = C::SHR[r][t];
            float x;
            if constexpr (s == 0) x = a - msg[e];
            else x = row_get(std::integral_constant<int, s>{}) - msg[e];
            if constexpr (QUANT) x = fminf(fmaxf(x, -qmax), qmax);
            msg[e] = x;
        });
    };
    if constexpr (APPB) {  // v2c of iteration 0 into the check frames
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) { gather_row(rr); });
    }
#else
    [[maybe_unused]] constexpr bool APPB = false;
#endif

    int it = 0;
    // QC_PH_MASK_IDLE (fixed count): the idle lanes (z >= Z: 10 of 64 at Z = 27) sit the iteration loop out,
    // EXEC-masked — no active lane ever reads them (rotation sources are active slots) — so they stop drawing power
    const bool loop_lane = !(QC_PH_MASK_IDLE && !EARLY) || z < Z;
    if (loop_lane) {
    for (; it + 1 < iters; ++it) {
#if QC_PH_LA && QC_PH_APPB
        if constexpr (APPB) {
            static_for<0, MB>([&](auto rr) __attribute__((always_inline)) { math_row(rr); });
            float T[2][DMX];
            if constexpr (QC_PH_APPB_LA) back_col(std::integral_constant<int, 0>{}, T[0]);
            static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
                constexpr int p = decltype(pp)::value;
                constexpr int j = lcol<C>(p);
                if constexpr (!QC_PH_APPB_LA) back_col(pp, T[p % 2]);
                else if constexpr (p + 1 < NB) back_col(std::integral_constant<int, p + 1>{}, T[(p + 1) % 2]);
                if constexpr (p % 4 == 0) {
                    Lg = lds_reload<4 * p, f4, 16>(Ls, lrow4);
                }
                float a = Lg[p % 4];
                static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) { a = a + T[p % 2][decltype(kk)::value]; });
                if (QUANT) a = fminf(fmaxf(a, -app_max), app_max);
                bcast_col(pp, a);
            });
            continue;
        }
#endif
#if QC_PH_LA
        if constexpr (!EARLY) {
            if constexpr (QC_PH_PRIO == 2 || QC_PH_PRIO == 3 || QC_PH_PRIO == 5) __builtin_amdgcn_s_setprio(1);
            if constexpr (QC_PH_PRIO == 1) __builtin_amdgcn_s_setprio(0);
            cn_phase_la();
            if constexpr (QC_PH_PRIO == 1) __builtin_amdgcn_s_setprio(1);
            if constexpr (QC_PH_PRIO == 2 || QC_PH_PRIO == 5) __builtin_amdgcn_s_setprio(0);
            static_for<0, (QC_PH_LA < NB ? QC_PH_LA : NB)>([&](auto pp) __attribute__((always_inline)) { rot_col(pp); });
            if constexpr (QC_PH_PRIO == 3) __builtin_amdgcn_s_setprio(0);
            static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
                constexpr int p = decltype(pp)::value;
                if constexpr (QC_PH_PRIO == 5) __builtin_amdgcn_s_setprio(1);
                if constexpr (p + QC_PH_LA < NB) rot_col(std::integral_constant<int, p + QC_PH_LA>{});
                if constexpr (QC_PH_PRIO == 5) __builtin_amdgcn_s_setprio(0);
                v2c_col(std::integral_constant<int, lcol<C>(p)>{}, sum_col(pp));
            });
            continue;
        }
#endif
        cn_phase();
        if constexpr (EARLY) {
            // APP_{it+1} of every column (kept until the syndrome verdict), hard-decision ballots
            float app[NB];
#if QC_PH_ES_ROWS
            // Row by row with an early exit (as the packed kernel's QC_PK_ES_ROWS): `cand` starts as the lane
            // groups (codewords) not yet done and loses each one whose row parity is nonzero; the scan stops once
            // neither codeword of the wave can still be satisfied — at low Eb/N0 after the first row.  The
            // ballots are taken at each use.  The decision equals the all-rows form's.
            static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
                constexpr int p = decltype(pp)::value;
                app[lcol<C>(p)] = vn_col(pp);
            });
            uint64_t cand = (G0 | G1) & ~done_groups;
            static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                constexpr int r = decltype(rr)::value;
                if (cand) {
                    uint64_t par = 0;
                    static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                        constexpr int t = decltype(tt)::value;
                        const uint64_t b = __ballot(app[C::COL[r][t]] <= thr2) & ACTIVE;
                        par ^= rot_lanes<Z, CPW, C::SHR[r][t]>(b);
                    });
                    par &= ACTIVE;
                    if (par & G0) cand &= ~G0;
                    if (par & G1) cand &= ~G1;
                }
            });
            const uint64_t fresh = cand;
#else
            uint64_t par[MB];
#pragma unroll
            for (int r = 0; r < MB; ++r) par[r] = 0;
            static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
                constexpr int p = decltype(pp)::value;
                constexpr int j = lcol<C>(p);
                app[j] = vn_col(pp);
                const uint64_t b = __ballot(app[j] <= thr2) & ACTIVE;
                static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                    constexpr int r = decltype(rr)::value;
                    constexpr int t = first_slot<C>(r, j);
                    if constexpr (t >= 0) par[r] ^= rot_lanes<Z, CPW, C::SHR[r][t]>(b);
                });
            });
            uint64_t unsat = 0;
#pragma unroll
            for (int r = 0; r < MB; ++r) unsat |= par[r];
            unsat &= ACTIVE;
            const uint64_t newly = ((unsat & G0) ? 0 : G0) | ((unsat & G1) ? 0 : G1);
            const uint64_t fresh = newly & ~done_groups;
#endif
            if (fresh) {
                // park the converged codeword's APP in its L row (L is no longer needed by it)
                if (fresh & G0) used_lo = it + 1;
                if (fresh & G1) used_hi = it + 1;
                if ((fresh >> lane) & 1ull) {
                    static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                        constexpr int j = decltype(jj)::value;
                        Ls[lrow + lpos<C>(j)] = app[j];
                    });
                }
                done_groups |= fresh;
                if (done_groups == (G0 | G1)) break;
            }
            static_for<0, NB>([&](auto jj) __attribute__((always_inline)) { v2c_col(jj, app[decltype(jj)::value]); });
        } else {
            static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
                constexpr int p = decltype(pp)::value;
                v2c_col(std::integral_constant<int, lcol<C>(p)>{}, vn_col(pp));
            });
        }
    }
    }  // loop_lane
    // last iteration (or early exit): outputs straight from the VN phase, column by column
    const bool early_exit = EARLY && done_groups == (G0 | G1);
    if (!early_exit && iters > 0) {
#if QC_PH_LA && QC_PH_APPB
        if constexpr (APPB) static_for<0, MB>([&](auto rr) __attribute__((always_inline)) { math_row(rr); });
        else cn_phase();
#else
        cn_phase();
#endif
    }
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int zo = tid & 31;
    const int64_t cwo = (((int64_t)blockIdx.x * blockDim.x + tid) >> 6) * CPW + ((tid >> 5) & 1);
    const bool parked = EARLY && ((done_groups >> (tid & 63)) & 1ull);
    const bool ok = zo < Z && cwo < B;
    static_for<0, NB>([&](auto pp) __attribute__((always_inline)) {
        constexpr int p = decltype(pp)::value;
        constexpr int j = lcol<C>(p);
        float a;
        if (iters > 0 && !early_exit) a = vn_col(pp);
        else a = Ls[lrow + p] + (iters == 0 ? 0.0f : -0.0f);  // iters == 0: APP_0 = L + (+0) (QUANT: clamped
                                                               // below); early exit: parked APP (x + -0 == x)
        if (QUANT && iters == 0) a = fminf(fmaxf(a, -app_max), app_max);
        if (parked) a = Ls[lrow + p];
        if (ok) {
            int t = zo + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            const int64_t o = cwo * N + j * Z + t;
            const float zz = 0.5f * a;
            if (bits) bits[o] = (uint8_t)(zz <= kZthrF32);
            if (soft) soft[o] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + expf(-zz));
        }
    });
    if (ok && zo == 0 && iters_used) iters_used[cwo] = ((tid >> 5) & 1) ? used_hi : used_lo;
}

// ---- tanh sum-product, register-resident (the reference's algorithm on-chip) ---------------------
// Messages in the variable frame, one VGPR per edge (c2v between iterations, v2c inside one), in log2 units.
// The operations are the oracle's (D, S) form and the generic kernels' (bp_vc.py:16-27, bp_cv.py:22-50
// evaluated as in common.h): per variable, v2c_t = copysign(exp2(-|fma(L, log2 e, S_t)|), .) with S_t the
// O(d) exclusive sum (vn_excl_sums); per check (cn_ds_row), each edge's log2(S/D) of the others' set, clamped
// to the reference's p clamp and to the caller's clamp; final z = fma(ascending sum, ln2/2, L/2).  Same device
// routines, so the values equal the generic GPU path's bit for bit.
#ifndef QC_SP_WAVES_PER_SIMD
#define QC_SP_WAVES_PER_SIMD 4
#endif
// QC_SP_SERIAL: each edge's exclusive sum / product chain starts after the previous edge's tanh / log
// output (an empty asm ties them): at most one chain in flight, instead of the scheduler interleaving a
// row's d chains and holding their partial products in registers.  Same operations, same order.  Fixed
// iteration count only: (648,1/2) 6.45 -> 6.79 M cw/s (A/B); the early-stop kernel is 0.5 % slower with it.
#ifndef QC_SP_SERIAL
#define QC_SP_SERIAL 1
#endif
#ifndef QC_SP_SERIAL_STRIDE
#define QC_SP_SERIAL_STRIDE 1  // with QC_SP_SERIAL: tie every k-th edge of a check row (k chains in flight)
#endif
#ifndef QC_SP_VN_OUT_TIE
#define QC_SP_VN_OUT_TIE 1  // the VC tie also pins each output (else the running sum alone: spills 50 VGPRs)
#endif
#ifndef QC_SP_SERIAL_VN_STRIDE
#define QC_SP_SERIAL_VN_STRIDE 1  // the same for the edges of a column
#endif
#ifndef QC_SP_SERIAL_ES_Z64
#define QC_SP_SERIAL_ES_Z64 1  // serial chains in the Z > 32 early-stop kernel: spill-free (6 VGPRs spilled before), same
#endif                         // speed ((1296,2/3) 8.42 vs 8.42 M cw/s, A/B)
#ifndef QC_SP_WAVES_PER_SIMD_EARLY
#define QC_SP_WAVES_PER_SIMD_EARLY 2  // 648 tanh-SP early stop 10.2 -> 12.1 M cw/s (A/B; 3 waves: 11.1)
#endif
// QC_SP_ADDR_MIN_USES (fixed iteration count): lane shifts used at least this many times per iteration get
// their ds_bpermute address computed once before the loop and held in a register (as k_qc_ms_ph), instead of
// a v_cndmask per rotation (the +4 rho folds into the ds_bpermute offset); 0 = off.  A/B (648,1/2) 50 it
// 12.73 -> 13.10 M cw/s, (1296,2/3) 20 it 15.43-15.63 -> 15.83-15.91 (4; 5: 13.00 / 15.61; 3 spills 51 VGPRs)
#ifndef QC_SP_ADDR_MIN_USES
#define QC_SP_ADDR_MIN_USES 4
#endif
#ifndef QC_SP_LPF
#define QC_SP_LPF 0  // VC phase: L of column j + QC_SP_LPF loaded before column j's chain (0: at its use).  A/B
#endif               // (profiles/r03/ab/ab_sp_lpf.txt): fixed count neutral ((648,1/2) 16.10 vs 16.05-16.09 M cw/s)
#ifndef QC_SP_LPF_EARLY
#define QC_SP_LPF_EARLY 3  // the same in the early-stop kernel (2 waves/SIMD): (648,1/2) 27.3-27.5 -> 28.1-28.5 M cw/s
#endif
#ifndef QC_SP_ES_ROWS
#define QC_SP_ES_ROWS 1  // early stop: syndrome row by row with an early exit, built in qc_es.hip (A/B
                         // profiles/r03/ab/ab_sp_esrows.txt: (648,1/2) 50 it 28.6 -> 29.2, (1296,2/3) 20 it 23.5 -> 24.8 M cw/s)
#endif
#ifndef QC_SP_GLA
#define QC_SP_GLA 0  // CV phase (fixed iteration count): row r + 1's gathers issued before row r's chains; A/B
                     // (648,1/2) 16.07 -> 15.73 M cw/s (the kernel is VALU-bound, not waiting on its gathers): off
#endif

// Early stop (EARLY): before iteration it >= 1, the hard decisions of z_it = 0.5 * (L + ascending sum of
// c2v) — the generic VN kernel's hb, same operations — are balloted per block column and rotated into
// each check's frame on the scalar unit (as k_qc_ms_st); a codeword whose syndrome is zero stops with
// iters_used = it and its z_it is parked in its own L region of LDS (its lanes keep computing for the
// wave's other codeword, discarded).  Bitwise equal to the generic path's early stop.
// PASS (the a == 1 rule, common.h cn_ds_row FIX): k_sp_zero_scan lists the waves whose codewords hold an
// exact-zero LLR (zlist: [0] = count, [1 ..] = wave ids, then one flag byte per wave, bit j = its codeword j —
// qc_sp_zflag); 1 = the plain
// loop for the unlisted waves (a listed one returns at once), 2 = the FIX loop for the listed waves (a small grid
// whose waves walk the list, on a second stream beside PASS 1: qc_sp_fork / qc_sp_join) — two kernels, so each
// keeps its own register allocation; 0 = the plain loop for every wave (QC_SP_FIXZ 0).
template <class C, bool EARLY, int PASS>
__device__ __forceinline__ void qc_sp_st_wave(int64_t wave_listed, const float* __restrict__ llr, int64_t B, int iters,
                                              float clamp, int flags, uint8_t* __restrict__ bits,
                                              float* __restrict__ soft, int32_t* __restrict__ iters_used,
                                              uint32_t* __restrict__ zlist) {
    constexpr int Z = C::Z, NB = C::NB, MB = C::MB, N = NB * Z;
    constexpr int NE = edge_off<C>(MB);
    static_assert(Z <= 64, "register kernel needs Z <= 64");
    constexpr int CPW = (Z <= 32) ? 2 : 1;
    const int lane = threadIdx.x & 63;
    const int half = (CPW == 2) ? (lane >> 5) : 0;
    const int z = (CPW == 2) ? (lane & 31) : lane;
    const int64_t wave = PASS == 2 ? wave_listed : ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t cw = wave * CPW + half;
    const bool valid = (z < Z) && (cw < B);
    const int zb = lane_zb<Z, CPW>(z);
    const int base4 = (half * 32 + zb) * 4;
    const int base4m = base4 - 4 * Z;
    if constexpr (PASS == 1) {  // a wave whose codewords hold an exact-zero LLR: the a == 1 rule's pass decodes it
        if (wave * CPW < B && qc_sp_zflag(zlist, B)[__builtin_amdgcn_readfirstlane((int)wave)]) return;
    }
    // lane rotations through a per-wave LDS row instead of ds_bpermute (see QC_PH_LDSROT)
    constexpr bool LDSROT = EARLY ? QC_SP_LDSROT_EARLY : QC_SP_LDSROT;
    __shared__ float Rw[LDSROT ? 256 : 1];
    const int wrow = LDSROT ? (int)(threadIdx.x & ~63u) * 4 : 0;
    if constexpr (LDSROT) {
        const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(&Rw[0]) + (unsigned)wrow);
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" ::"s"(m0) : "memory");
    }
    auto xfer = [&](int addr, float x) __attribute__((always_inline)) {
        if constexpr (LDSROT) {
            asm volatile("ds_write_addtid_b32 %0" ::"v"(x) : "memory");
            return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(Rw) + wrow + addr);
        } else {
            return bperm(addr, x);
        }
    };
    // rotation addresses: "read lane (z + rho) mod Z of my group", one register per frequently used shift
    constexpr int ADDR_MIN = EARLY ? 0 : QC_SP_ADDR_MIN_USES;
    int ra[Z];
    static_for<1, Z>([&](auto rr) __attribute__((always_inline)) {
        constexpr int rho = decltype(rr)::value;
        if constexpr (ADDR_MIN > 0 && rot_uses<C>(rho) >= ADDR_MIN)
            ra[rho] = sel_lanes<wrap_mask<Z, CPW>(Z - rho)>(base4, base4m) + 4 * rho;
    });
    (void)ra;
    auto raddr = [&](auto rr) __attribute__((always_inline)) {
        constexpr int rho = decltype(rr)::value;
        if constexpr (ADDR_MIN > 0 && rot_uses<C>(rho) >= ADDR_MIN) return ra[rho];
        else return sel_lanes<wrap_mask<Z, CPW>(Z - rho)>(base4, base4m) + 4 * rho;
    };
    __shared__ float Ls[(sp_tpb<EARLY>() / 64) * CPW * N];
    const int lbase = ((threadIdx.x >> 6) * CPW + half) * N + z;
    const int lbase4 = lbase * 4;  // bytes (lds_reload)
    {
        const int64_t cwbase = valid ? cw * N : 0;
        const float vmask = valid ? 1.0f : 0.0f;
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            int t = z + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            const float x = llr[cwbase + j * Z + (valid ? t : 0)] * vmask;
            if (z < Z) Ls[lbase + j * Z] = -x;  // L = -llr (bp.py:47)
        });
    }
    float msg[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) msg[e] = 0.0f;
    const float cmax2 = sp_cmax2(clamp);  // check outputs in log2 units (common.h)
    constexpr uint64_t ACTIVE = lane_range_mask<Z, CPW>(0, Z);
    uint64_t done_groups = 0;  // lane masks of converged codewords (CPW == 2)
    int used_lo = iters, used_hi = iters;

    // QC_SP_MASK_IDLE (fixed count): idle lanes (z >= Z) sit the iteration loop out, EXEC-masked (as QC_PH_MASK_IDLE)
    const bool loop_lane = !(QC_SP_MASK_IDLE && !EARLY) || z < Z;
    constexpr bool FIX = PASS == 2;
    // the rule applies per codeword (common.h): this lane's codeword's bit of the unit's flag
    uint32_t fixm = 0x7fffffffu;
    if constexpr (FIX) fixm = ((qc_sp_zflag(zlist, B)[wave] >> half) & 1u) ? 0x7fffffffu : 0u;
    if (loop_lane)
    for (int it = 0; it < iters; ++it) {
        if constexpr (EARLY) {
            if (it > 0) {
                // z of column j from the c2v of the previous iteration (the epilogue's association)
                auto zcol = [&](auto jj) __attribute__((always_inline)) {
                    constexpr int j = decltype(jj)::value;
                    float S = 0.0f;
                    static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) {
                        S += msg[col_edge<C>(j, decltype(kk)::value)];
                    });
                    return sp_z(lds_reload<4 * j * Z, float>(Ls, lbase4), S);
                };
#if QC_SP_ES_ROWS
                // row by row with an early exit (as the min-sum kernels): the columns' hard decisions packed in
                // one register, then each row's parity from ballots of its columns' bits until no codeword of
                // the wave can still be satisfied
                static_assert(NB <= 32, "one hard-decision bit per block column in a 32-bit word");
                uint32_t hd = 0;
                static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                    constexpr int j = decltype(jj)::value;
                    hd |= Num<float>::bit(zcol(jj)) ? (1u << j) : 0u;
                });
                constexpr uint64_t GA = lane_range_mask<Z, 1>(0, Z), GB = (CPW == 2) ? (GA << 32) : 0;
                uint64_t cand = (GA | GB) & ~done_groups;
                static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                    constexpr int r = decltype(rr)::value;
                    if (cand) {
                        uint64_t par = 0;
                        static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                            constexpr int t = decltype(tt)::value;
                            const uint64_t b = __ballot((hd >> C::COL[r][t]) & 1u) & ACTIVE;
                            par ^= rot_lanes<Z, CPW, C::SHR[r][t]>(b);
                        });
                        if (par & GA) cand &= ~GA;
                        if constexpr (CPW == 2) {
                            if (par & GB) cand &= ~GB;
                        }
                    }
                });
                const uint64_t unsat = (GA | GB) & ~cand;
#else
                uint64_t par[MB];
#pragma unroll
                for (int r = 0; r < MB; ++r) par[r] = 0;
                static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                    constexpr int j = decltype(jj)::value;
                    const uint64_t b = __ballot(Num<float>::bit(zcol(jj))) & ACTIVE;
                    static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                        constexpr int r = decltype(rr)::value;
                        constexpr int t = first_slot<C>(r, j);
                        if constexpr (t >= 0) par[r] ^= rot_lanes<Z, CPW, C::SHR[r][t]>(b);
                    });
                });
                uint64_t unsat = 0;
#pragma unroll
                for (int r = 0; r < MB; ++r) unsat |= par[r];
                unsat &= ACTIVE;
#endif
                if constexpr (CPW == 1) {
                    if (unsat == 0) {  // the wave's codeword converged: its c2v are the output's
                        used_lo = it;
                        break;
                    }
                } else {
                    constexpr uint64_t G0 = lane_range_mask<Z, 1>(0, Z), G1 = G0 << 32;
                    const uint64_t newly = ((unsat & G0) ? 0 : G0) | ((unsat & G1) ? 0 : G1);
                    const uint64_t fresh = newly & ~done_groups;
                    if (fresh) {
                        if (fresh & G0) used_lo = it;
                        if (fresh & G1) used_hi = it;
                        if ((fresh >> lane) & 1ull) {
                            static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                                constexpr int j = decltype(jj)::value;
                                const float zz = zcol(jj);
                                Ls[lbase + j * Z] = zz;  // parked z (its L is no longer needed)
                            });
                        }
                        done_groups |= fresh;
                        if (done_groups == (G0 | G1)) break;
                    }
                }
            }
        }
        // VC + tanh in the variable frame: c2v -> v2c in place
        if constexpr (!EARLY && QC_SP_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        // L of column j + LPF is loaded before column j's chain (its address asm precedes the chain's ties),
        // so its LDS latency hides under the chains instead of a lgkmcnt(0) wait per column
        constexpr int LPF = EARLY ? QC_SP_LPF_EARLY : QC_SP_LPF;
        float Lq[LPF > 0 ? LPF : 1];
        static_for<0, LPF>([&](auto qq) __attribute__((always_inline)) {
            constexpr int q = decltype(qq)::value;
            if constexpr (q < NB) Lq[q] = lds_reload<4 * q * Z, float>(Ls, lbase4);
        });
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            constexpr int dj = col_deg<C>(j);
            float L;
            if constexpr (LPF > 0) {
                L = Lq[j % LPF];
                if constexpr (j + LPF < NB) Lq[j % LPF] = lds_reload<4 * (j + LPF) * Z, float>(Ls, lbase4);
            } else {
                L = lds_reload<4 * j * Z, float>(Ls, lbase4);
            }
            constexpr bool TIE = QC_SP_SERIAL && (!EARLY || (QC_SP_SERIAL_ES_Z64 && Z > 32));
            vn_excl_sums<dj, TIE ? QC_SP_SERIAL_VN_STRIDE : 0>(
                [&](auto kk) __attribute__((always_inline)) { return msg[col_edge<C>(j, decltype(kk)::value)]; },
                [&](auto kk, float S) __attribute__((always_inline)) {
                    constexpr int k = decltype(kk)::value;
                    constexpr int e = col_edge<C>(j, k);
                    msg[e] = vn_signed_a(sp_vn_arg(L, S));  // the (D, S) form's VC output (common.h)
                    if constexpr (TIE && QC_SP_VN_OUT_TIE && (k + 1) % QC_SP_SERIAL_VN_STRIDE == 0)
                        SP_TIE("+v"(msg[e]));  // next edge's chain starts after this output
                });
        });
        // CV in the check frame: gather v2c, exclusive products, log, clamp, scatter c2v back
        if constexpr (!EARLY && QC_SP_PRIO == 2) __builtin_amdgcn_s_setprio(0);
#if QC_SP_GLA
        // gathers issued one row ahead, in place on msg[] (as k_qc_ms_ph's lookahead): row r + 1's rotations
        // are in flight while row r's chains run
        auto gather_sp = [&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int s = C::SHR[r][t];
                if constexpr (s != 0) msg[edge_off<C>(r) + t] = xfer(raddr(std::integral_constant<int, s>{}), msg[edge_off<C>(r) + t]);
            });
        };
        if constexpr (!EARLY) gather_sp(std::integral_constant<int, 0>{});
#endif
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            constexpr int e0 = edge_off<C>(r);
            float g[d];
#if QC_SP_GLA
            constexpr bool GLA = !EARLY;
            if constexpr (GLA && r + 1 < MB) gather_sp(std::integral_constant<int, r + 1>{});
#else
            constexpr bool GLA = false;
#endif
            if constexpr (!EARLY && QC_SP_PRIO == 1) __builtin_amdgcn_s_setprio(1);
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int s = C::SHR[r][t];
                if constexpr (s == 0 || GLA) {
                    g[t] = msg[e0 + t];
                } else {
                    g[t] = xfer(raddr(std::integral_constant<int, s>{}), msg[e0 + t]);
                }
            });
            if constexpr (!EARLY && QC_SP_PRIO == 1) __builtin_amdgcn_s_setprio(0);
            cn_ds_row<d, (QC_SP_SERIAL && (!EARLY || (QC_SP_SERIAL_ES_Z64 && Z > 32))) ? QC_SP_SERIAL_STRIDE : 0, 0, DS_BLOCK,
                      FIX>(g, cmax2, fixm);
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int s = C::SHR[r][t];
                if constexpr (s == 0) {
                    msg[e0 + t] = g[t];
                } else {
                    msg[e0 + t] = xfer(raddr(std::integral_constant<int, Z - s>{}), g[t]);
                }
            });
        });
    }
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int zo = (CPW == 2) ? (tid & 31) : (tid & 63);
    const int64_t wo = PASS == 2 ? wave : (((int64_t)blockIdx.x * blockDim.x + tid) >> 6);
    const int64_t cwo = wo * CPW + ((CPW == 2) ? ((tid >> 5) & 1) : 0);
    const bool parked = EARLY && CPW == 2 && ((done_groups >> (tid & 63)) & 1ull);
    if (zo < Z && cwo < B) {
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            constexpr int dj = col_deg<C>(j);
            float S = 0.0f;
            static_for<0, dj>([&](auto kk) __attribute__((always_inline)) { S += msg[col_edge<C>(j, decltype(kk)::value)]; });
            const float zz = parked ? Ls[lbase + j * Z] : sp_z(Ls[lbase + j * Z], S);
            int t = zo + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            const int64_t o = cwo * N + j * Z + t;
            if (bits) bits[o] = (uint8_t)Num<float>::bit(zz);
            if (soft) soft[o] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + Num<float>::exp_(-zz));
        });
        if (zo == 0 && iters_used) iters_used[cwo] = (CPW == 2 && ((tid >> 5) & 1)) ? used_hi : used_lo;
    }
}

template <class C, bool EARLY, int PASS = 1>
__global__ __launch_bounds__(256, EARLY ? QC_SP_WAVES_PER_SIMD_EARLY : QC_SP_WAVES_PER_SIMD) void k_qc_sp_st(const float* __restrict__ llr, int64_t B, int iters,
                                                                       float clamp, int flags, uint8_t* __restrict__ bits,
                                                                       float* __restrict__ soft, int32_t* __restrict__ iters_used,
                                                                       uint32_t* __restrict__ zlist) {
    if constexpr (PASS == 2) {  // the listed waves, walked by this grid's waves
        const uint32_t n = zlist[0];
        const uint32_t nw = gridDim.x * (blockDim.x >> 6);
        for (uint32_t i = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6); i < n; i += nw)
            qc_sp_st_wave<C, EARLY, 2>(__builtin_amdgcn_readfirstlane(zlist[1 + i]), llr, B, iters, clamp, flags, bits,
                                       soft, iters_used, zlist);
    } else {
        qc_sp_st_wave<C, EARLY, PASS>(0, llr, B, iters, clamp, flags, bits, soft, iters_used, zlist);
    }
}

#ifndef QC_ES_TU
#define QC_ES_TU 1  // the float early-stop min-sum and tanh-SP register kernels come from qc_es.hip (0: instantiated here)
#endif
#if QC_TU_ES
// qc_es.hip includes this file with QC_TU_ES = 1 and builds it with the default scheduler: it instantiates
// only the early-stop register kernels (k_qc_ms_ph<C, false, true, N> for Z <= 32, k_qc_ms_st<C, false,
// true, N> above, k_qc_sp_st<C, true>), whose row-wise syndromes (QC_PH/ST/SP_ES_ROWS) run faster there than under the
// iterative-ILP scheduler of the fixed-count kernels (A/B profiles/r03/ab/ab_ph_esrows.txt, ab_st_esrows.txt)
template <class C>
static int launch_ms_es(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft, int32_t* used,
                        hipStream_t st) {
    constexpr int CPW = (C::Z <= 32) ? 2 : 1;
    const int64_t waves = (B + CPW - 1) / CPW;
    const int tpb = st_tpb<true>();
    const unsigned blocks = (unsigned)((waves + tpb / 64 - 1) / (tpb / 64));
    const float* x = (const float*)llr;
    float* sf = (float*)soft;
    const int norm = (p.alpha != 1.0f ? NORM_ALPHA : 0) | (p.beta != 0.0f ? NORM_BETA : 0);
#define FE(N)                                                                                                     \
    do {                                                                                                          \
        if constexpr (C::Z <= 32)                                                                                 \
            k_qc_ms_ph<C, false, true, N><<<blocks, tpb, 0, st>>>(x, B, p.iters, p.clamp, p.alpha, p.beta, 0.f, 0.f, 1.f, p.flags, bits, sf, used); \
        else                                                                                                      \
            k_qc_ms_st<C, false, true, N><<<blocks, tpb, 0, st>>>(x, B, p.iters, p.clamp, p.alpha, p.beta, 0.f, 0.f, 1.f, p.flags, bits, sf, used); \
    } while (0)
    switch (norm) {
        case NORM_PLAIN: FE(NORM_PLAIN); break;
        case NORM_ALPHA: FE(NORM_ALPHA); break;
        case NORM_BETA: FE(NORM_BETA); break;
        default: FE(NORM_BOTH);
    }
#undef FE
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "qc kernel launch: %s", hipGetErrorString(e));
    return LDPC_OK;
}
template <class C>
static int launch_sp_es(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft, int32_t* used,
                        hipStream_t st) {
    constexpr int CPW = (C::Z <= 32) ? 2 : 1;
    const int64_t waves = (B + CPW - 1) / CPW;
    const int tpb = sp_tpb<true>();
    const unsigned blocks = (unsigned)((waves + tpb / 64 - 1) / (tpb / 64));
    if constexpr (QC_SP_FIXZ) {
        uint32_t* zl = qc_sp_zlist();
        hipStream_t s2;
        if (const int rc = qc_sp_fork((const float*)llr, B, C::NB * C::Z, CPW, st, &s2)) return rc;
        k_qc_sp_st<C, true, 2><<<qc_sp_pass2_grid(blocks), tpb, 0, s2>>>((const float*)llr, B, p.iters, p.clamp, p.flags, bits, (float*)soft, used, zl);
        k_qc_sp_st<C, true, 1><<<blocks, tpb, 0, st>>>((const float*)llr, B, p.iters, p.clamp, p.flags, bits, (float*)soft, used, zl);
        if (const int rc = qc_sp_join(st)) return rc;
    } else {
        k_qc_sp_st<C, true, 0><<<blocks, tpb, 0, st>>>((const float*)llr, B, p.iters, p.clamp, p.flags, bits, (float*)soft, used, nullptr);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "qc kernel launch: %s", hipGetErrorString(e));
    return LDPC_OK;
}
int qc_launch_ms_es_wifi648_12(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                               int32_t* used, hipStream_t st) {
    return p.algo == LDPC_ALGO_TANH_SP ? launch_sp_es<Wifi648_12>(llr, B, p, bits, soft, used, st)
                                       : launch_ms_es<Wifi648_12>(llr, B, p, bits, soft, used, st);
}
int qc_launch_ms_es_wifi1296_23(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                                int32_t* used, hipStream_t st) {
    return p.algo == LDPC_ALGO_TANH_SP ? launch_sp_es<Wifi1296_23>(llr, B, p, bits, soft, used, st)
                                       : launch_ms_es<Wifi1296_23>(llr, B, p, bits, soft, used, st);
}
#else
// float early-stop min-sum (qc_es.hip)
int qc_launch_ms_es_wifi648_12(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                               int32_t* used, hipStream_t st);
int qc_launch_ms_es_wifi1296_23(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                                int32_t* used, hipStream_t st);

// packed quantized kernels (qc_pk.hip)
int qc_launch_qms_pk_wifi648_12(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                                int32_t* used, hipStream_t st);
int qc_launch_qms_pk_wifi1296_23(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                                 int32_t* used, hipStream_t st);
#ifndef QC_PACKED
#define QC_PACKED 1  // quantized min-sum for Z <= 64 runs the packed fp16 kernel (0: float-register kernels, A/B)
#endif

// sliced kernels for Z > 64 (qc_sl.hip)
int qc_launch_sl_wifi1944_56(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                              int32_t* used, hipStream_t st);

#ifndef QC_STORED
#define QC_STORED 1  // min-sum launches use k_qc_ms_st (fixed or early stop); 0: compressed k_qc_ms (A/B builds)
#endif
#ifndef QC_PHASED
#define QC_PHASED 1  // Z <= 32 min-sum: the phased kernel k_qc_ms_ph (0: k_qc_ms_st, A/B builds)
#endif

template <class C>
static int launch_ms(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft, int32_t* used,
                     hipStream_t st) {
    constexpr int CPW = (C::Z <= 32) ? 2 : 1;
    const int64_t waves = (B + CPW - 1) / CPW;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    const bool es = (p.flags & LDPC_F_EARLY_STOP) != 0;
    const int tpb_st = es ? st_tpb<true>() : st_tpb<false>(), tpb_sp = es ? sp_tpb<true>() : sp_tpb<false>();
    const unsigned blocks_st = (unsigned)((waves + tpb_st / 64 - 1) / (tpb_st / 64));
    const unsigned blocks_sp = (unsigned)((waves + tpb_sp / 64 - 1) / (tpb_sp / 64));
    const float* x = (const float*)llr;
    float* sf = (float*)soft;
    if (p.algo == LDPC_ALGO_TANH_SP) {
        if constexpr (QC_ES_TU != 0) {
            if (es) {  // qc_es.hip
                if constexpr (std::is_same_v<C, Wifi648_12>) return qc_launch_ms_es_wifi648_12(llr, B, p, bits, soft, used, st);
                else return qc_launch_ms_es_wifi1296_23(llr, B, p, bits, soft, used, st);
            }
        } else {
            if (es) k_qc_sp_st<C, true, 0><<<blocks_sp, tpb_sp, 0, st>>>(x, B, p.iters, p.clamp, p.flags, bits, sf, used, nullptr);
        }
        if (!es) {
            if constexpr (QC_SP_FIXZ) {  // the plain pass, then the a == 1 rule's pass for waves with a zero LLR
                uint32_t* zl = qc_sp_zlist();
                hipStream_t s2;
                if (const int rc = qc_sp_fork(x, B, C::NB * C::Z, CPW, st, &s2)) return rc;
                k_qc_sp_st<C, false, 2><<<qc_sp_pass2_grid(blocks_sp), tpb_sp, 0, s2>>>(x, B, p.iters, p.clamp, p.flags, bits, sf, used, zl);
                k_qc_sp_st<C, false, 1><<<blocks_sp, tpb_sp, 0, st>>>(x, B, p.iters, p.clamp, p.flags, bits, sf, used, zl);
                if (const int rc = qc_sp_join(st)) return rc;
            } else {
                k_qc_sp_st<C, false, 0><<<blocks_sp, tpb_sp, 0, st>>>(x, B, p.iters, p.clamp, p.flags, bits, sf, used, nullptr);
            }
        }
    } else if (p.algo == LDPC_ALGO_QMIN_SUM && QC_PACKED != 0) {
        // two codewords per lane in packed fp16 (qc_pk.hip)
        if constexpr (std::is_same_v<C, Wifi648_12>) return qc_launch_qms_pk_wifi648_12(llr, B, p, bits, soft, used, st);
        else if constexpr (std::is_same_v<C, Wifi1296_23>) return qc_launch_qms_pk_wifi1296_23(llr, B, p, bits, soft, used, st);
        else return set_error(LDPC_EUNSUPPORTED, "no packed quantized kernel for %s", C::NAME);
    } else if (p.algo == LDPC_ALGO_QMIN_SUM) {
#if !QC_PACKED  // the float-register quantized kernels (A/B builds only)
        const float qm = (float)p.qmax, am = (float)p.app_max, b = (float)(int)p.beta, qi = 1.0f / p.qstep;
#define QL(E, N)                                                                                                  \
    do {                                                                                                          \
        if constexpr (QC_PHASED != 0 && C::Z <= 32)                                                             \
            k_qc_ms_ph<C, true, E, N><<<blocks_st, tpb_st, 0, st>>>(x, B, p.iters, qm, 1.0f, b, qm, am, qi, p.flags, bits, sf, used); \
        else if constexpr (QC_STORED != 0)                                                                        \
            k_qc_ms_st<C, true, E, N><<<blocks_st, tpb_st, 0, st>>>(x, B, p.iters, qm, 1.0f, b, qm, am, qi, p.flags, bits, sf, used); \
        else                                                                                                      \
            k_qc_ms<C, true, E, N><<<blocks, 256, 0, st>>>(x, B, p.iters, qm, 1.0f, b, qm, am, qi, p.flags, bits, sf, used); \
    } while (0)
        if (b != 0.0f) { if (es) QL(true, NORM_BETA); else QL(false, NORM_BETA); }
        else           { if (es) QL(true, NORM_PLAIN); else QL(false, NORM_PLAIN); }
#undef QL
#endif
    } else {
        if constexpr (QC_PHASED != 0 && QC_STORED != 0 && QC_ES_TU != 0) {
            if (es) {
                if constexpr (std::is_same_v<C, Wifi648_12>) return qc_launch_ms_es_wifi648_12(llr, B, p, bits, soft, used, st);
                else return qc_launch_ms_es_wifi1296_23(llr, B, p, bits, soft, used, st);
            }
        }
        const int norm = (p.alpha != 1.0f ? NORM_ALPHA : 0) | (p.beta != 0.0f ? NORM_BETA : 0);
#define FL(E, N)                                                                                                  \
    do {                                                                                                          \
        if constexpr (E && QC_PHASED != 0 && QC_STORED != 0 && QC_ES_TU != 0) {                              \
        } else if constexpr (QC_PHASED != 0 && C::Z <= 32)                                                      \
            k_qc_ms_ph<C, false, E, N><<<blocks_st, tpb_st, 0, st>>>(x, B, p.iters, p.clamp, p.alpha, p.beta, 0.f, 0.f, 1.f, p.flags, bits, sf, used); \
        else if constexpr (QC_STORED != 0)                                                                        \
            k_qc_ms_st<C, false, E, N><<<blocks_st, tpb_st, 0, st>>>(x, B, p.iters, p.clamp, p.alpha, p.beta, 0.f, 0.f, 1.f, p.flags, bits, sf, used); \
        else                                                                                                      \
            k_qc_ms<C, false, E, N><<<blocks, 256, 0, st>>>(x, B, p.iters, p.clamp, p.alpha, p.beta, 0.f, 0.f, 1.f, p.flags, bits, sf, used); \
    } while (0)
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
#define SPEC_SL(C, F) {C::MB, C::NB, C::Z, &C::COL[0][0], &C::SH[0][0], &C::DEG[0], C::MAXDC, C::NAME, &F}
static const QCSpec kSpecs[] = {SPEC(Wifi648_12), SPEC(Wifi1296_23), SPEC_SL(Wifi1944_56, qc_launch_sl_wifi1944_56)};
#undef SPEC_SL
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
    if (p.algo == LDPC_ALGO_TANH_SP) return true;  // Z <= 64: k_qc_sp_st; Z = 81: k_qc_sp_sl (both with early stop)
    return p.algo == LDPC_ALGO_MIN_SUM || p.algo == LDPC_ALGO_QMIN_SUM;
}

// tanh-SP: the zero-LLR list of the two-pass kernels (qc_sp_zlist, qc_sp_zflag): a count, at most one id per
// codeword, then one flag byte per codeword
size_t qc_workspace(const QCSpec*, int64_t B, const ldpc_params& p) {
    return (p.algo == LDPC_ALGO_TANH_SP && QC_SP_FIXZ) ? (size_t)((4 * (B + 1) + B + 255) & ~(int64_t)255) : 0;
}

uint32_t*& qc_sp_zlist() {
    static thread_local uint32_t* f = nullptr;
    return f;
}

// one wave per unit of `cpu` (<= 8) consecutive codewords (n LLRs each, row-major): flag = bit j set when codeword j
// of the unit holds an exact-zero LLR (+-0; the a == 1 rule is per codeword, common.h), the unit listed once when any
// is.  Reads the batch's LLRs once (B n 4 bytes) so that the a == 1 rule's units can run beside the plain pass
// instead of after it.
__global__ __launch_bounds__(256) void k_sp_zero_scan(const float* __restrict__ llr, int64_t B, int n, int cpu,
                                                      int64_t units, uint32_t* __restrict__ zlist) {
    const int64_t u = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (u >= units) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const int64_t c0 = u * cpu, c1 = (c0 + cpu < B) ? c0 + cpu : B;
    uint32_t mask = 0;
    for (int64_t c = c0; c < c1; ++c) {
        const float* p = llr + c * n;
        bool z = false;
        int64_t i0 = 0;
        if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
            const float4* p4 = reinterpret_cast<const float4*>(p);
            const int64_t n4 = n >> 2;
            for (int64_t i = lane; i < n4; i += 64) {
                const float4 v = p4[i];
                z |= (v.x == 0.0f) | (v.y == 0.0f) | (v.z == 0.0f) | (v.w == 0.0f);
            }
            i0 = n4 << 2;
        }
        for (int64_t i = i0 + lane; i < n; i += 64) z |= p[i] == 0.0f;
        mask |= (__ballot(z) != 0 ? 1u : 0u) << (c - c0);
    }
    if (lane == 0) {
        qc_sp_zflag(zlist, B)[u] = (uint8_t)mask;
        if (mask) zlist[1 + atomicAdd(zlist, 1u)] = (uint32_t)u;
    }
}

namespace {
// Auxiliary streams for the forked decodes (the a == 1 rule's pass, the IRA path's Infinity-Cache chunks): kAux
// streams and their fork / join events per (host thread, device, CALLER stream) — keyed by the caller's stream so
// that decodes on different caller streams never share an auxiliary stream (no false dependence of one caller's join
// on another's fork, and a graph capture open on stream A never absorbs a decode issued on stream B), and per host
// thread so that no two threads interleave one set's fork / join.  At most kAuxSets sets per thread (the least
// recently used one outside any open graph capture is destroyed — hipStreamDestroy lets its pending work finish);
// a thread's sets are destroyed when it exits.
constexpr int kAux = 3;
constexpr int kAuxSets = 16;
struct Aux {
    int dev = -1;
    hipStream_t caller = nullptr;
    uint64_t used = 0;  // LRU stamp
    hipStream_t s[kAux] = {};
    hipEvent_t fork = nullptr, join[kAux] = {};
    void release() {
        for (int i = 0; i < kAux; ++i) {
            if (s[i]) (void)hipStreamDestroy(s[i]);
            if (join[i]) (void)hipEventDestroy(join[i]);
            s[i] = nullptr;
            join[i] = nullptr;
        }
        if (fork) (void)hipEventDestroy(fork);
        fork = nullptr;
        dev = -1;
        caller = nullptr;
    }
    bool create() {
        if (hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess) {
            fork = nullptr;
            return false;
        }
        for (int i = 0; i < kAux; ++i) {
            if (hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking) != hipSuccess) {
                s[i] = nullptr;
                return false;
            }
            if (hipEventCreateWithFlags(&join[i], hipEventDisableTiming) != hipSuccess) {
                join[i] = nullptr;
                return false;
            }
        }
        return true;
    }
};
struct AuxPool {
    Aux set[kAuxSets];
    uint64_t clock = 0;
    ~AuxPool() {
        for (Aux& a : set)
            if (a.dev >= 0) a.release();
    }
};
bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}
bool any_capturing(const Aux& a) {
    for (int i = 0; i < kAux; ++i)
        if (a.s[i] && capturing(a.s[i])) return true;
    return false;
}
Aux* aux_get(hipStream_t caller) {
    static thread_local AuxPool pool;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    Aux* lru = nullptr;
    for (Aux& a : pool.set) {
        if (a.dev == dev && a.caller == caller) {
            a.used = ++pool.clock;
            return &a;
        }
    }
    // evict the least recently used set whose streams are not part of an open graph capture (destroying one
    // would invalidate that capture); none free: the caller gets an error, not a broken graph
    for (Aux& a : pool.set)
        if ((!lru || a.used < lru->used) && (a.dev < 0 || !any_capturing(a))) lru = &a;
    if (!lru) return nullptr;
    if (lru->dev >= 0) lru->release();
    if (!lru->create()) {
        lru->release();
        return nullptr;
    }
    lru->dev = dev;
    lru->caller = caller;
    lru->used = ++pool.clock;
    return lru;
}
}  // namespace

int aux_fork(hipStream_t st, hipStream_t* s2, int n) {
    Aux* a = aux_get(st);
    if (!a || n < 1 || n > kAux) return set_error(LDPC_EHIP, "auxiliary streams unavailable");
    // an auxiliary stream still inside a capture the caller is not part of (a capture that ended abnormally) would
    // record this decode into that graph
    if (!capturing(st))
        for (int i = 0; i < n; ++i)
            if (capturing(a->s[i])) return set_error(LDPC_EHIP, "auxiliary stream is inside another stream's graph capture");
    if (hipEventRecord(a->fork, st) != hipSuccess) return set_error(LDPC_EHIP, "auxiliary stream: fork failed");
    for (int i = 0; i < n; ++i) {
        if (hipStreamWaitEvent(a->s[i], a->fork, 0) != hipSuccess)
            return set_error(LDPC_EHIP, "auxiliary stream: fork failed");
        s2[i] = a->s[i];
    }
    return LDPC_OK;
}

int aux_join(hipStream_t st, int n) {
    Aux* a = aux_get(st);
    if (!a || n < 1 || n > kAux) return set_error(LDPC_EHIP, "auxiliary streams unavailable");
    for (int i = 0; i < n; ++i)
        if (hipEventRecord(a->join[i], a->s[i]) != hipSuccess || hipStreamWaitEvent(st, a->join[i], 0) != hipSuccess)
            return set_error(LDPC_EHIP, "auxiliary stream: join failed");
    return LDPC_OK;
}

int qc_sp_fork(const float* llr, int64_t B, int n, int cpu, hipStream_t st, hipStream_t* s2) {
    uint32_t* zl = qc_sp_zlist();
    if (!zl) return set_error(LDPC_EHIP, "tanh-SP zero-LLR pass: no workspace");
    if (cpu < 1 || cpu > 8) return set_error(LDPC_EHIP, "tanh-SP zero-LLR pass: %d codewords per unit (flag byte holds 8)", cpu);
    if (hipMemsetAsync(zl, 0, 4, st) != hipSuccess) return set_error(LDPC_EHIP, "zero-LLR list reset failed");
    const int64_t units = (B + cpu - 1) / cpu;
    k_sp_zero_scan<<<(unsigned)((units + 3) / 4), 256, 0, st>>>(llr, B, n, cpu, units, zl);
    return aux_fork(st, s2);
}

int qc_sp_join(hipStream_t st) { return aux_join(st); }

int qc_decode(const QCSpec* s, const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
              int32_t* used, char* ws, hipStream_t st) {
    qc_sp_zlist() = (uint32_t*)ws;
    const int rc = s->launch_ms(llr, B, p, bits, soft, used, st);
    qc_sp_zlist() = nullptr;
    return rc;
}
#endif  // QC_TU_ES

}  // namespace ldpc
