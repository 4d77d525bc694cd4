// qc_sl.hip — sliced register kernels for quasi-cyclic codes with Z > 64 (802.11n Z = 81), gfx950.
#include "qc_sl_sp.h"

// ---- sliced register kernels for Z > 64 (802.11n Z = 81) -----------------------------------------
// The lifting index is split into S slots of ZL = Z / S <= 32 lanes: a unit of S waves decodes two
// codewords (lane halves), wave k holding frame positions zc = l + ZL*k of every block column/row.  Each
// wave keeps its slot's messages in VGPRs; a circulant with rotation rho != 0 moves values between
// waves, so it is exchanged through LDS: every lane stores its value at positions zc and zc + Z of a
// per-circulant row [half][2Z] (two copies, so the reader's (zc + rho) mod Z needs no wrap), a barrier,
// and the reader loads position zc + rho — one base VGPR per lane, every offset an instruction
// immediate.  Rotation-0 circulants (the lane frames make 30 of 79 so for (1944,5/6)) stay in registers.
// Per block row: store v2c, barrier, gather, check update, store c2v, barrier, scatter (two buffers).
// The tanh-SP kernel and the shared helpers are in qc_sl_sp.h.

namespace ldpc {

// Min-sum, stored messages in the CHECK frame (fixed iterations or early stop, float or 5-bit quantized).
// Per iteration: every wave publishes APP_it of its slot (two copies per position) to LDS, one barrier;
// per block row: gather APP_it into the check frame (registers for rotation 0), v2c = APP - c2v_old,
// two-minimum + sign product, new c2v kept in registers; rotation-!=0 c2v go through one LDS row buffer
// (barrier before the stores, barrier before the loads) and are added into APP_{it+1} in ascending row
// order.  The arithmetic is k_qc_ms_st's / the oracle's operation for operation (bit-exact).  Early stop:
// the syndrome of APP_it falls out of the gather (parity of the gathered hard decisions, one ballot per
// row); the S waves' verdicts meet in LDS at the last row's barrier, so the whole unit agrees on which
// of its two codewords converged (frozen: APP_it kept, iters_used = it).
template <class C, bool QUANT, bool EARLY, int NORM>
__global__ __launch_bounds__(C::S * 64) __attribute__((amdgpu_waves_per_eu(QC_SL_WAVES_PER_SIMD)))
void k_qc_ms_sl(const float* __restrict__ llr, int64_t B, int iters, float clamp, float alpha, float beta, float qmax,
                float app_max, float qinv, int flags, uint8_t* __restrict__ bits, float* __restrict__ soft,
                int32_t* __restrict__ iters_used) {
    constexpr int Z = C::Z, S = C::S, ZL = Z / S, NB = C::NB, MB = C::MB, N = NB * Z;
    constexpr int NE = edge_off<C>(MB), NT = nz_max<C>(), ROW = 2 * 2 * Z;
    static_assert(S > 1 && Z % S == 0 && ZL <= 32, "sliced kernel: Z = S * ZL, ZL <= 32");
    __shared__ float Xa[NB * ROW];  // APP_it of every block column, [j][half][2Z]
    __shared__ float Xc[NT * ROW];  // one block row's rotated c2v
    __shared__ uint32_t Fl[2 * S];  // early stop: (slot, half) has an unsatisfied check
    const int k = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    const int64_t cw = (int64_t)blockIdx.x * 2 + h;
    const bool live = l < ZL;
    const bool valid = live && cw < B;
    const int zc = live ? l + ZL * k : (QC_SL_IDLE_ALIAS ? ZL * k : 0);  // idle lanes: see qc_sl_sp.h
    const int xb = h * 2 * Z + zc;
    float Lr[NB], app[NB];
    {
        const int64_t base = valid ? cw * N : 0;
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            int t = zc + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            float x = valid ? llr[base + j * Z + t] : 0.0f;
            if (QUANT) x = fminf(fmaxf(rintf(x * qinv), -qmax), qmax);
            Lr[j] = -x;
            app[j] = QUANT ? fminf(fmaxf(-x, -app_max), app_max) : -x + 0.0f;  // APP_0 = L + (+0) c2v: -0 -> +0
        });
    }
    float msg[NE];  // c2v of every edge, check frame
#pragma unroll
    for (int e = 0; e < NE; ++e) msg[e] = 0.0f;
    const float thr2n = __uint_as_float(__float_as_uint(2.0f * kZthrF32) - 1u);  // next float above 2*ZTHR
    const int64_t cw0 = (int64_t)blockIdx.x * 2;
    bool done0 = cw0 >= B, done1 = cw0 + 1 >= B;  // a missing codeword counts as converged
    int used0 = iters, used1 = iters;

    for (int it = 0; it < iters; ++it) {
        if (live) {
            static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                constexpr int j = decltype(jj)::value;
                Xa[j * ROW + xb] = app[j];
                Xa[j * ROW + xb + Z] = app[j];
            });
        }
        __syncthreads();
        float nap[NB];
        uint64_t unsat = 0;
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            constexpr int e0 = edge_off<C>(r);
            float v[d];
            float mn1, mn2;
            uint32_t par = 0;
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int j = C::COL[r][t], s = C::SHR[r][t];
                const float a = Xa[j * ROW + xb + s];  // from LDS even for s == 0: app[] is dead during the rows
                if constexpr (EARLY) par ^= __float_as_uint(a - thr2n);
                float x = a - msg[e0 + t];
                if constexpr (QUANT) x = fminf(fmaxf(x, -qmax), qmax);
                v[t] = x;
            });
            two_min(v, mn1, mn2);
            if constexpr (EARLY) unsat |= __ballot((int)par < 0);
            const uint32_t tot = xor_all(v) & 0x80000000u;
            const float M1 = __uint_as_float(__float_as_uint(mag_of<NORM>(mn1, alpha, beta, clamp)) ^ tot);
            const float M2 = __uint_as_float(__float_as_uint(mag_of<NORM>(mn2, alpha, beta, clamp)) ^ tot);
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                // |v| == min1 picks the min slot; ties imply min2 == min1 (bit-exact, see k_qc_ms)
                const float mg = (fabsf(v[t]) == mn1) ? M2 : M1;
                msg[e0 + t] = __uint_as_float(__float_as_uint(mg) ^ (__float_as_uint(v[t]) & 0x80000000u));
            });
            if constexpr (EARLY && r == MB - 1) {
                if (lane == 0) {
                    Fl[2 * k] = (uint32_t)((unsat & 0xffffffffull) != 0);
                    Fl[2 * k + 1] = (uint32_t)((unsat >> 32) != 0);
                }
            }
            if constexpr (nz_count<C>(r) > 0) {
                __syncthreads();  // the previous row's rotated c2v have been read by every wave
                if (live) {
                    static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                        constexpr int t = decltype(tt)::value;
                        if constexpr (C::SHR[r][t] != 0) {
                            constexpr int o = nz_index<C>(r, t) * ROW;
                            Xc[o + xb] = msg[e0 + t];
                            Xc[o + xb + Z] = msg[e0 + t];
                        }
                    });
                }
                __syncthreads();
            } else if constexpr (r == MB - 1) {
                __syncthreads();  // every wave's Xa gathers are done before the next iteration's stores
            }
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int j = C::COL[r][t], s = C::SHR[r][t];
                const float cr = (s == 0) ? msg[e0 + t] : Xc[nz_index<C>(r, t) * ROW + xb + (Z - s)];
                if constexpr (first_row<C>(j) == r) nap[j] = Lr[j];
                nap[j] = nap[j] + cr;
            });
        });
        if constexpr (EARLY) {
            uint32_t u0 = 0, u1 = 0;
#pragma unroll
            for (int q = 0; q < S; ++q) {
                u0 |= Fl[2 * q];
                u1 |= Fl[2 * q + 1];
            }
            if (it > 0 && !done0 && u0 == 0) { done0 = true; used0 = it; }
            if (it > 0 && !done1 && u1 == 0) { done1 = true; used1 = it; }
            const bool frozen = h ? done1 : done0;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const float nx = QUANT ? fminf(fmaxf(nap[j], -app_max), app_max) : nap[j];
                app[j] = frozen ? Xa[j * ROW + xb] : nx;  // Xa still holds APP_it
            }
            if (done0 && done1) break;
        } else {
#pragma unroll
            for (int j = 0; j < NB; ++j) app[j] = QUANT ? fminf(fmaxf(nap[j], -app_max), app_max) : nap[j];
        }
    }
    if (valid) {
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            int t = zc + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            const int64_t o = cw * N + j * Z + t;
            const float zz = 0.5f * app[j];
            if (bits) bits[o] = (uint8_t)(zz <= kZthrF32);
            if (soft) soft[o] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + expf(-zz));
        });
        if (k == 0 && l == 0 && iters_used) iters_used[cw] = h ? used1 : used0;
    }
}

int qc_launch_sp_sl_es_wifi1944_56(const float* llr, int64_t B, const ldpc_params& p, uint8_t* bits, float* soft,
                                   int32_t* used, hipStream_t st);

template <class C>
static int launch_sl(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft, int32_t* used,
                     hipStream_t st) {
    const unsigned blocks = (unsigned)((B + 1) / 2);  // one unit of S waves per codeword pair
    const dim3 tb(C::S * 64);
    const bool es = (p.flags & LDPC_F_EARLY_STOP) != 0;
    const float* x = (const float*)llr;
    float* sf = (float*)soft;
    if (p.algo == LDPC_ALGO_TANH_SP) {
        if (es) {
            static_assert(std::is_same_v<C, Wifi1944_56>, "one sliced code");
            qc_launch_sp_sl_es_wifi1944_56(x, B, p, bits, sf, used, st);
        } else if (QC_SL_SP_RS) {  // the plain pass, then the a == 1 rule's pass for units with a zero LLR
            hipStream_t s2 = st;
            if (QC_SP_FIXZ) {
                if (const int rc = qc_sp_fork(x, B, C::NB * C::Z, 2, st, &s2)) return rc;
                k_qc_sp_rs<C, 2><<<qc_sp_pass2_grid(blocks), tb, 0, s2>>>(x, B, p.iters, p.clamp, p.flags, bits, sf, used, qc_sp_zlist());
            }
            k_qc_sp_rs<C, QC_SP_FIXZ ? 1 : 0><<<blocks, tb, 0, st>>>(x, B, p.iters, p.clamp, p.flags, bits, sf, used, qc_sp_zlist());
            if (QC_SP_FIXZ)
                if (const int rc = qc_sp_join(st)) return rc;
        } else {
            hipStream_t s2 = st;
            if (QC_SP_FIXZ) {
                if (const int rc = qc_sp_fork(x, B, C::NB * C::Z, 2, st, &s2)) return rc;
                k_qc_sp_sl<C, false, 2><<<qc_sp_pass2_grid(blocks), tb, 0, s2>>>(x, B, p.iters, p.clamp, p.flags, bits, sf, used, qc_sp_zlist());
            }
            k_qc_sp_sl<C, false, QC_SP_FIXZ ? 1 : 0><<<blocks, tb, 0, st>>>(x, B, p.iters, p.clamp, p.flags, bits, sf, used, qc_sp_zlist());
            if (QC_SP_FIXZ)
                if (const int rc = qc_sp_join(st)) return rc;
        }
    } else if (p.algo == LDPC_ALGO_QMIN_SUM) {
        const float qm = (float)p.qmax, am = (float)p.app_max, b = (float)(int)p.beta, qi = 1.0f / p.qstep;
#define QL(E, N) k_qc_ms_sl<C, true, E, N><<<blocks, tb, 0, st>>>(x, B, p.iters, qm, 1.0f, b, qm, am, qi, p.flags, bits, sf, used)
        if (b != 0.0f) { if (es) QL(true, NORM_BOTH); else QL(false, NORM_BOTH); }
        else           { if (es) QL(true, NORM_PLAIN); else QL(false, NORM_PLAIN); }
#undef QL
    } else {
        // NORM_BOTH is bit-identical to the alpha-only / beta-only forms for their cases (qc_common.h)
        const bool plain = p.alpha == 1.0f && p.beta == 0.0f;
#define FL(E, N) k_qc_ms_sl<C, false, E, N><<<blocks, tb, 0, st>>>(x, B, p.iters, p.clamp, p.alpha, p.beta, 0.f, 0.f, 1.f, p.flags, bits, sf, used)
        if (plain) { if (es) FL(true, NORM_PLAIN); else FL(false, NORM_PLAIN); }
        else       { if (es) FL(true, NORM_BOTH); else FL(false, NORM_BOTH); }
#undef FL
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "qc kernel launch: %s", hipGetErrorString(e));
    return LDPC_OK;
}

int qc_launch_sl_wifi1944_56(const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
                              int32_t* used, hipStream_t st) {
    return launch_sl<Wifi1944_56>(llr, B, p, bits, soft, used, st);
}

}  // namespace ldpc
