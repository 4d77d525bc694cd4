// qc_sl_sp.h — the sliced tanh-SP kernel for Z > 64 (802.11n Z = 81) and the sliced kernels' helpers.
// Included by qc_sl.hip (fixed iteration count, iterative-ILP scheduler) and qc_sl_es.hip (early stop,
// default scheduler: with the ILP scheduler the early-stop variant needs > 256 VGPRs and spills).
#pragma once
#include "qc_common.h"

namespace ldpc {

template <class C>
constexpr int nz_count(int r) {  // circulants of row r with a nonzero rotation
    int c = 0;
    for (int t = 0; t < C::DEG[r]; ++t) c += (C::SHR[r][t] != 0);
    return c;
}
template <class C>
constexpr int nz_index(int r, int t) {
    int c = 0;
    for (int u = 0; u < t; ++u) c += (C::SHR[r][u] != 0);
    return c;
}
template <class C>
constexpr int nz_max() {
    int m = 1;
    for (int r = 0; r < C::MB; ++r) m = nz_count<C>(r) > m ? nz_count<C>(r) : m;
    return m;
}

#ifndef QC_SL_WAVES_PER_SIMD
#define QC_SL_WAVES_PER_SIMD 3
#endif
// Per variant (fixed iteration count / EARLY) — occupancy, exchange buffers, where L lives; A/B on the box
// (profiles/r02/ab/): fixed 1.47 -> 1.86 M cw/s with serial chains, one buffer, L from global, 4 waves;
// early stop 2.27 -> 2.50 M cw/s with serial chains at 2 waves (3 waves / one buffer / L in global: 2.46).
#ifndef QC_SL_SP_WAVES_PER_SIMD
#define QC_SL_SP_WAVES_PER_SIMD 4
#endif
#ifndef QC_SL_SP_WAVES_PER_SIMD_EARLY
#define QC_SL_SP_WAVES_PER_SIMD_EARLY 2
#endif

// Early stop (EARLY): before iteration it >= 1, every lane sums its columns' c2v (ascending, the generic VN
// kernel's operations) into z_it = 0.5 * (L + sum) and publishes the hard decision to LDS (two copies per
// position, like the exchange rows); each check lane then XORs the decisions of its edges' variables (the
// gather's positions) and the unit's waves pool one ballot per (slot, codeword) in LDS.  A codeword whose
// syndrome is zero writes its outputs from z_it right there (iters_used = it) and is skipped at the end;
// the unit leaves the loop when both of its codewords are done.  Bitwise equal to the generic path.
// QC_SL_SP_SERIAL_CN = k > 0: every k-th edge's exclusive product (CN) / sum (VN) chain starts after the previous edge's
// log / tanh output (an empty asm ties them), so one chain is in flight instead of a row's 20 partial
// products held in registers: 195 -> 112 VGPRs for the same operations in the same order.
// QC_SL_SP_COMPACT: one exchange buffer for v2c and c2v (a third barrier per row instead of a second
// buffer).  QC_SL_SP_L: where L lives — 0 VGPRs, 1 LDS, 2 re-read from global memory (an L2 hit) at every
// use.  Fixed-count kernel: one buffer + L in global = 26 KB of LDS per unit, 112 VGPRs: five units
// (15 waves) per CU instead of two.
#ifndef QC_SL_POS_STRIDE
// lane l of slot wave k holds frame position S*l + k (1) instead of l + ZL*k (0): a rotation by c reads positions
// (S*l + k + c) mod Z = S*((l + q) mod ZL) + r, whose LDS banks (a/4 mod 32) are distinct for odd S, so no access
// of the rotated-circulant slots conflicts; with contiguous positions every window that wraps past Z conflicted
// (round 4: SQ_LDS_BANK_CONFLICT 21 % of the resident kernel's LDS cycles).  A relabelling: bitwise the same.
#define QC_SL_POS_STRIDE 1
#endif
#ifndef QC_SL_IDLE_ALIAS
#define QC_SL_IDLE_ALIAS 1  // idle lanes read at their wave's first position (0: at position 0, round 2)
#endif
#ifndef QC_SL_SP_SERIAL_CN
#define QC_SL_SP_SERIAL_CN 1
#endif
#ifndef QC_SL_SP_SERIAL_ROW
#define QC_SL_SP_SERIAL_ROW QC_SL_SP_SERIAL_CN  // the check rows' ties alone (cn_ds_row's SERIAL)
#endif
#ifndef QC_SL_SP_COMPACT
#define QC_SL_SP_COMPACT 1
#endif
#ifndef QC_SL_SP_COMPACT_EARLY
#define QC_SL_SP_COMPACT_EARLY 0
#endif
#ifndef QC_SL_SP_L
#define QC_SL_SP_L 2
#endif
#ifndef QC_SL_SP_L_EARLY
#define QC_SL_SP_L_EARLY 0
#endif
// QC_SL_SP_LPF (L from global memory): the VN phase loads L of column j + 1 before column j's chains.  The
// serial-chain asm statements order memory operations, so without it every column waits out an L2 hit.
#ifndef QC_SL_SP_LPF
#define QC_SL_SP_LPF 0  // A/B: 1.874 vs 1.887 M cw/s, -0.8 % (profiles/r02/ab/ab_lpf.txt): the other waves hide it
#endif

#ifndef QC_SL_DIAG_NOBAR
#define QC_SL_DIAG_NOBAR 0  // DIAGNOSTIC BUILD ONLY (wrong results): no row-exchange barriers, to price them
#endif
__device__ __forceinline__ void sl_barrier() {
    if constexpr (!QC_SL_DIAG_NOBAR) __syncthreads();
}

// PASS: as k_qc_sp_st's (qc.hip) — 1 = the plain loop for the units k_sp_zero_scan did not list, 2 = the a == 1
// rule's loop for the listed units, 0 = the plain loop for every unit.  A unit = one workgroup's two codewords;
// unit_listed is the unit of PASS 2 (the others use the block index).
template <class C, bool EARLY, int PASS>
__device__ __forceinline__ void qc_sp_sl_unit(uint32_t unit_listed, const float* __restrict__ llr, int64_t B, int iters,
                                              float clamp, int flags, uint8_t* __restrict__ bits,
                                              float* __restrict__ soft, int32_t* __restrict__ iters_used,
                                              uint32_t* __restrict__ zlist) {
    const int64_t unit = PASS == 2 ? (int64_t)unit_listed : (int64_t)blockIdx.x;
    if constexpr (PASS == 1) {
        if (unit * 2 < B && qc_sp_zflag(zlist, B)[unit]) return;  // listed: the a == 1 rule's pass (uniform)
    }
    constexpr int Z = C::Z, S = C::S, ZL = Z / S, NB = C::NB, MB = C::MB, N = NB * Z;
    constexpr int NE = edge_off<C>(MB), NT = nz_max<C>(), ROW = 2 * 2 * Z;  // floats per exchanged circulant
    static_assert(S > 1 && Z % S == 0 && ZL <= 32, "sliced kernel: Z = S * ZL, ZL <= 32");
    constexpr bool CMP = EARLY ? QC_SL_SP_COMPACT_EARLY : QC_SL_SP_COMPACT;
    constexpr int LM = EARLY ? QC_SL_SP_L_EARLY : QC_SL_SP_L;
    __shared__ float Xv[NT * ROW], Xc2[CMP ? 1 : NT * ROW];
    float* const Xc = CMP ? Xv : Xc2;
    __shared__ float Lsh[LM == 1 ? 2 * NB * Z : 1];  // L of both codewords: [half][j][position]
    const int k = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // slot of this wave
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    const int64_t cw = unit * 2 + h;
    const bool live = l < ZL;                // lane carries a frame position
    const bool valid = live && cw < B;       // ... of a real codeword
    // idle lanes (l >= ZL) alias this wave's first position for reads (they never store): an exchange read is
    // served per 32-lane half with bank = (address / 4) mod 32, and aliased to position 0 (round 2) the idle
    // lanes of waves k = 1, 2 read a distinct address on a bank their active lanes use — one extra LDS cycle
    // per read; repeating an active lane's address of their own wave is a broadcast instead.
    const int p0 = QC_SL_POS_STRIDE ? k : ZL * k;  // this wave's first position
    const int zc = live ? (QC_SL_POS_STRIDE ? S * l + k : l + ZL * k) : (QC_SL_IDLE_ALIAS ? p0 : 0);
    const int xb = h * 2 * Z + zc;           // this lane's position in an exchange row
    // L = -llr (bp.py:47) of this lane's variable in every block column
    const float* const lp = llr + (valid ? cw * N : 0);
    const int lb = h * NB * Z + zc;
    float Lr[LM == 0 ? NB : 1];
    auto Lr_at = [&](int j) __attribute__((always_inline)) {
        if constexpr (LM == 2) {
            int z = zc;
            asm volatile("" : "+v"(z));  // re-read at every use (an L2 hit), not hoisted into registers
            int t = z + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            return valid ? -lp[j * Z + t] : 0.0f;
        } else if constexpr (LM == 1) {
            int a = lb;
            asm volatile("" : "+v"(a));  // re-read every iteration, not hoisted into registers
            return Lsh[a + j * Z];
        } else {
            return Lr[j];
        }
    };
    if constexpr (LM != 2) {
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            int t = zc + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            const float x = valid ? -lp[j * Z + t] : 0.0f;
            if constexpr (LM == 1) {
                if (live) Lsh[lb + j * Z] = x;
            } else {
                Lr[j] = x;
            }
        });
    }
    __syncthreads();  // the L rows of LM == 1
    float msg[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) msg[e] = 0.0f;
    const float cmax2 = sp_cmax2(clamp);  // check outputs in log2 units (common.h)
    // outputs of this lane's codeword from z of every column (end of the loop, or at convergence)
    auto emit = [&](auto zfun) __attribute__((always_inline)) {
        if (valid) {
            static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                constexpr int j = decltype(jj)::value;
                const float zz = zfun(jj);
                int t = zc + C::PHI[j];
                t -= (t >= Z) ? Z : 0;
                const int64_t o = cw * N + j * Z + t;
                if (bits) bits[o] = (uint8_t)Num<float>::bit(zz);
                if (soft) soft[o] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + Num<float>::exp_(-zz));
            });
        }
    };
    auto zsum = [&](auto jj) __attribute__((always_inline)) {  // z = 0.5 * (L + ascending sum of c2v)
        constexpr int j = decltype(jj)::value;
        float Ssum = 0.0f;
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) { Ssum += msg[col_edge<C>(j, decltype(kk)::value)]; });
        return sp_z(Lr_at(j), Ssum);
    };
    constexpr int HROW = 2 * 2 * Z;  // hard decisions: [j][half][2Z] bytes
    __shared__ uint8_t Hb[EARLY ? NB * HROW : 1];
    __shared__ uint32_t Fl[2 * S];
    __shared__ float Zp[EARLY ? 2 * NB * Z : 1];  // parked z of converged codewords, [half][j][position]
    const int64_t cwp = unit * 2;
    bool done0 = cwp >= B, done1 = cwp + 1 >= B;  // a missing codeword counts as converged
    int used0 = iters, used1 = iters;

    constexpr bool FIX = PASS == 2;
    // the rule applies per codeword (common.h): this lane's codeword's bit of the unit's flag
    uint32_t fixm = 0x7fffffffu;
    if constexpr (FIX) fixm = ((qc_sp_zflag(zlist, B)[unit] >> h) & 1u) ? 0x7fffffffu : 0u;
    for (int it = 0; it < iters; ++it) {
        if constexpr (EARLY) {
            if (it > 0) {
                if (live) {
                    static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                        constexpr int j = decltype(jj)::value;
                        const uint8_t b = (uint8_t)Num<float>::bit(zsum(jj));
                        Hb[j * HROW + xb] = b;
                        Hb[j * HROW + xb + Z] = b;
                    });
                }
                __syncthreads();
                uint32_t un = 0;  // some check of this lane's codeword position is unsatisfied
                static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
                    constexpr int r = decltype(rr)::value;
                    uint32_t par = 0;
                    static_for<0, C::DEG[r]>([&](auto tt) __attribute__((always_inline)) {
                        constexpr int t = decltype(tt)::value;
                        par ^= Hb[C::COL[r][t] * HROW + xb + C::SHR[r][t]];
                    });
                    un |= par;
                    asm volatile("" : "+v"(un));  // one row's loads in flight at a time (register budget)
                });
                const uint64_t bu = __ballot(live && un != 0);
                if (lane == 0) {
                    Fl[2 * k] = (uint32_t)((bu & 0xffffffffull) != 0);
                    Fl[2 * k + 1] = (uint32_t)((bu >> 32) != 0);
                }
                __syncthreads();
                uint32_t u0 = 0, u1 = 0;
#pragma unroll
                for (int q = 0; q < S; ++q) {
                    u0 |= Fl[2 * q];
                    u1 |= Fl[2 * q + 1];
                }
                const bool new0 = !done0 && u0 == 0, new1 = !done1 && u1 == 0;
                if (new0) used0 = it;
                if (new1) used1 = it;
                if (live && (h ? new1 : new0)) {  // park z_it, this codeword's output (emitted after the loop)
                    static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
                        constexpr int j = decltype(jj)::value;
                        float Ssum = 0.0f;
                        asm volatile("" : "+v"(Ssum));  // not CSE'd with the syndrome pass above
                        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) {
                            Ssum += msg[col_edge<C>(j, decltype(kk)::value)];
                        });
                        Zp[(h * NB + j) * Z + zc] = sp_z(Lr_at(j), Ssum);
                    });
                }
                done0 |= new0;
                done1 |= new1;
                if (done0 && done1) break;
                // (Hb / Fl are rewritten only after this iteration's row barriers: no barrier needed here)
            }
        }
        // VC + tanh in the variable frame (as k_qc_sp_st)
        constexpr bool LPF = LM == 2 && QC_SL_SP_LPF;
        float Lnext = LPF ? Lr_at(0) : 0.0f;
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            constexpr int dj = col_deg<C>(j);
            const float Lj = LPF ? Lnext : Lr_at(j);
            if constexpr (LPF && j + 1 < NB) Lnext = Lr_at(j + 1);  // in flight during this column's chains
            vn_excl_sums<dj, QC_SL_SP_SERIAL_CN>(  // O(d) exclusive sums (common.h), k chains in flight
                [&](auto kk) __attribute__((always_inline)) { return msg[col_edge<C>(j, decltype(kk)::value)]; },
                [&](auto kk, float Ssum) __attribute__((always_inline)) {
                    constexpr int q = decltype(kk)::value;
                    constexpr int e = col_edge<C>(j, q);
                    msg[e] = vn_signed_a(sp_vn_arg(Lj, Ssum));  // the (D, S) form's VC output (common.h)
                    if constexpr (QC_SL_SP_SERIAL_CN > 0 && (q + 1) % QC_SL_SP_SERIAL_CN == 0)
                        SP_TIE("+v"(msg[e]));  // next edge's chain starts after this output
                });
        });
        // CV per block row through the LDS exchange
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            constexpr int e0 = edge_off<C>(r);
            if (live) {
                static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                    constexpr int t = decltype(tt)::value;
                    if constexpr (C::SHR[r][t] != 0) {
                        constexpr int o = nz_index<C>(r, t) * ROW;
                        Xv[o + xb] = msg[e0 + t];
                        Xv[o + xb + Z] = msg[e0 + t];
                    }
                });
            }
            sl_barrier();
            float g[d];
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int s = C::SHR[r][t];
                if constexpr (s == 0) g[t] = msg[e0 + t];
                else g[t] = Xv[nz_index<C>(r, t) * ROW + xb + s];
            });
            cn_ds_row<d, QC_SL_SP_SERIAL_ROW, 0, DS_BLOCK, FIX>(g, cmax2, fixm);  // O(d) exclusive sets (common.h)
            if constexpr (CMP) sl_barrier();  // every wave has read this row's v2c before the buffer takes its c2v
            if (live) {
                static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                    constexpr int t = decltype(tt)::value;
                    if constexpr (C::SHR[r][t] != 0) {
                        constexpr int o = nz_index<C>(r, t) * ROW;
                        Xc[o + xb] = g[t];
                        Xc[o + xb + Z] = g[t];
                    }
                });
            }
            sl_barrier();
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                constexpr int s = C::SHR[r][t];
                if constexpr (s == 0) msg[e0 + t] = g[t];
                else msg[e0 + t] = Xc[nz_index<C>(r, t) * ROW + xb + (Z - s)];
            });
            if constexpr (CMP) sl_barrier();  // ... and its c2v before the next row's v2c lands in the buffer
        });
    }
    if (EARLY && (h ? done1 : done0)) {
        emit([&](auto jj) __attribute__((always_inline)) { return Zp[(h * NB + decltype(jj)::value) * Z + zc]; });
    } else {
        emit(zsum);
    }
    if (valid && k == 0 && l == 0 && iters_used) iters_used[cw] = h ? used1 : used0;
}

template <class C, bool EARLY, int PASS = 1>
__global__ __launch_bounds__(C::S * 64)
__attribute__((amdgpu_waves_per_eu(EARLY ? QC_SL_SP_WAVES_PER_SIMD_EARLY : QC_SL_SP_WAVES_PER_SIMD)))
void k_qc_sp_sl(const float* __restrict__ llr, int64_t B, int iters, float clamp, int flags,
                uint8_t* __restrict__ bits, float* __restrict__ soft, int32_t* __restrict__ iters_used,
                uint32_t* __restrict__ zlist) {
    if constexpr (PASS == 2) {  // the listed units, walked by this grid's workgroups
        const uint32_t n = zlist[0];
        for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
            qc_sp_sl_unit<C, EARLY, 2>(__builtin_amdgcn_readfirstlane(zlist[1 + i]), llr, B, iters, clamp, flags, bits,
                                       soft, iters_used, zlist);
            __syncthreads();  // the unit's last LDS reads before the next unit's writes
        }
    } else {
        qc_sp_sl_unit<C, EARLY, PASS>(0, llr, B, iters, clamp, flags, bits, soft, iters_used, zlist);
    }
}

// ---- resident sliced tanh-SP (config [2]: 802.11n (1944,5/6), Z = 81) ------------------------------
// k_qc_sp_sl above keeps every message in VGPRs and exchanges the rotated circulants' values through an LDS
// row per block row: three or four barriers per block row (16 per iteration), SQ_WAIT_ANY 0.39.  Here the
// messages of the ROTATED circulants live in LDS for the whole decode, one 32-bit slot per (edge, position),
// updated in place: the VN phase reads every column's c2v, forms its v2c and writes them back at the same
// slots; a barrier; the CN phase reads every row's v2c, forms its c2v and writes them back; a barrier — two
// barriers per iteration.  Each slot is touched by exactly one lane in each phase (its variable's owner in
// the VN phase, its check's owner in the CN phase), so in place is race-free between the two barriers.
// Rotation-0 circulants (30 of 79) keep their messages in VGPRs as before.
// Addressing without a per-access modulo: circulant (r, t) with rotation rho = Q*a + b (Q = 9 for Z = 81)
// stores check position p at slot (p + Q*a) mod Z of its row of Z floats; the check's owner (position p)
// reads slot (p + Q*a) mod Z and the variable's owner (position z = p + rho) slot (z - b) mod Z — the same
// slot.  Each lane precomputes its byte address for the Z/Q values of a and the Q values of b once (17
// VGPRs for Z = 81, where every rotation would need its own: 42); the circulant's row offset rides in the
// ds instruction's immediate.  LDS: 49 rotated circulants x 2 codewords x 81 x 4 B = 31.0 KiB per unit of
// three waves, five units (15 waves) per CU, as the register-exchange kernel.  Arithmetic operation for
// operation that kernel's (bitwise equal results; tests/test_gpu_parity.py).
#ifndef QC_SL_SP_RS
#define QC_SL_SP_RS 1
#endif
#ifndef QC_RS_WAVES_PER_SIMD
#define QC_RS_WAVES_PER_SIMD 4
#endif
#ifndef QC_RS_SERIAL
#define QC_RS_SERIAL 1  // the VN chains' ties (vn_excl_sums' TIE)
#endif
#ifndef QC_RS_SERIAL_ROW
#define QC_RS_SERIAL_ROW 1  // the check rows' ties (cn_ds_row's SERIAL); 2: 59 VGPRs spilled
#endif
#ifndef QC_RS_ADDR_OPAQUE
#define QC_RS_ADDR_OPAQUE 0  // 1: address VGPRs through an empty asm at each use (a v_mov each: 4.09 vs 4.28 M cw/s)
#endif
#ifndef QC_RS_DS_BLOCK
// check rows (d = 20) in blocks of this many edges (common.h cn_ds_row; bitwise the same outputs).  20: one block,
// no shared suffix pass — with the fma join 4.96 -> 5.30 M cw/s (1,279 -> 1,182 VALU per wave-iteration); 16: 5.18,
// 14: 5.13 (no spill); 7: 4.86 (profiles/r04/ab/ab_rs2.txt).  At 20, five VGPRs (values set before the iteration
// loop and read after it) go to scratch around the loop — no scratch access inside it (tests/test_kernel_resources.py);
// recomputing the output indices after the loop moved a spill INTO the loop instead.
#define QC_RS_DS_BLOCK 20
#endif
#ifndef QC_RS_PRIO
// 1: s_setprio 1 over the latency-bound VN phase (short chains between LDS loads), 0 over the issue-bound CN phase,
// so a SIMD issues the VN waves' loads as soon as they are ready and fills the gaps with CN work: 4.35 -> 4.67 M
// cw/s (A/B profiles/r04/ab/ab_rs.txt); 2: the reverse, 4.25; 3: as 1, and the CN phase's row gathers at 1 too
#define QC_RS_PRIO 1
#endif
#ifndef QC_RS_MASK_IDLE
#define QC_RS_MASK_IDLE 0  // A/B -1.5 % (profiles/r04/ab/ab_mask.txt)
#endif
#ifndef QC_RS_IDLE_DUP
#define QC_RS_IDLE_DUP 0  // 1: idle lanes l >= 27 shadow lane l - 27 (same loads, same values) and store too: no exec branches
#endif
#ifndef QC_RS_ROW_LAG
#define QC_RS_ROW_LAG 0  // 1: the check rows' ties lag one edge (two edges' outputs in flight, common.h)
#endif
#ifndef QC_RS_VPF
#define QC_RS_VPF 0  // 1: the VN phase loads column j + 1's messages before column j's chains and stores
#endif
#ifndef QC_RS_CPF
#define QC_RS_CPF 0  // k > 0: the CN phase loads the last k edges of row r + 1 (read first) before row r's chains
#endif
#ifndef QC_RS_L
#define QC_RS_L 0  // where L lives: 0 VGPRs (loaded once), 2 re-read from global memory at every use (3.64 vs 4.09)
#endif

template <class C>
constexpr int rs_rot_index(int r, int t) {  // index of circulant (r, t) among the rotated ones, check order
    int c = 0;
    for (int q = 0; q < C::MB; ++q)
        for (int u = 0; u < C::DEG[q]; ++u) {
            if (q == r && u == t) return c;
            c += (C::SHR[q][u] != 0);
        }
    return -1;
}
template <class C>
constexpr int rs_zero_index(int r, int t) {  // index of circulant (r, t) among the rotation-0 ones
    int c = 0;
    for (int q = 0; q < C::MB; ++q)
        for (int u = 0; u < C::DEG[q]; ++u) {
            if (q == r && u == t) return c;
            c += (C::SHR[q][u] == 0);
        }
    return -1;
}
template <class C>
constexpr int rs_rot_total() {
    return rs_rot_index<C>(C::MB - 1, C::DEG[C::MB - 1] - 1) + (C::SHR[C::MB - 1][C::DEG[C::MB - 1] - 1] != 0);
}
template <class C>
constexpr int rs_max_col_deg() {
    int m = 1;
    for (int j = 0; j < C::NB; ++j) m = col_deg<C>(j) > m ? col_deg<C>(j) : m;
    return m;
}
template <int Z>
constexpr int rs_q() {  // the smallest Q with Q * Q >= Z (9 for 81)
    int q = 1;
    while (q * q < Z) ++q;
    return q;
}

// QC_RS_DIAG_NOBAR (DIAGNOSTIC BUILDS ONLY, wrong results): the two barriers per iteration removed, to price them
#ifndef QC_RS_DIAG_NOBAR
#define QC_RS_DIAG_NOBAR 0
#endif
template <class C, int PASS>  // PASS, unit_listed: as qc_sp_sl_unit's
__device__ __forceinline__ void qc_sp_rs_unit(uint32_t unit_listed, const float* __restrict__ llr, int64_t B, int iters,
                                              float clamp, int flags, uint8_t* __restrict__ bits,
                                              float* __restrict__ soft, int32_t* __restrict__ iters_used,
                                              uint32_t* __restrict__ zlist) {
    const int64_t unit = PASS == 2 ? (int64_t)unit_listed : (int64_t)blockIdx.x;
    if constexpr (PASS == 1) {
        if (unit * 2 < B && qc_sp_zflag(zlist, B)[unit]) return;  // listed: the a == 1 rule's pass (uniform)
    }
    constexpr int Z = C::Z, S = C::S, ZL = Z / S, NB = C::NB, MB = C::MB, N = NB * Z;
    constexpr int NE = edge_off<C>(MB), NR = rs_rot_total<C>(), N0 = NE - NR;
    constexpr int Q = rs_q<Z>(), NA = (Z - 1) / Q + 1;
    constexpr int CROW = 2 * Z * 4;  // bytes per rotated circulant: [half][position]
    static_assert(S > 1 && Z % S == 0 && ZL <= 32, "sliced kernel: Z = S * ZL, ZL <= 32");
    static_assert(NR * CROW < 65536, "circulant offsets ride in the 16-bit ds offset");
    __shared__ float X[NR * 2 * Z];
    char* const Xb = reinterpret_cast<char*>(X);
    const int k = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // slot of this wave
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    const int64_t cw = unit * 2 + h;
    const bool live = l < ZL;                // lane carries a frame position (stores are live lanes only)
    const bool valid = live && cw < B;
    // idle lanes read at their wave's first position (a broadcast, see k_qc_sp_sl) and never store; with
    // QC_RS_IDLE_DUP they shadow lane l - ZL instead — the same loads, so the same values, written to the same
    // slots by the same instruction — and the stores need no exec mask
    auto pos_of = [&](int ll) { return QC_SL_POS_STRIDE ? S * ll + k : ll + ZL * k; };  // see QC_SL_POS_STRIDE
    const int zc = live ? pos_of(l) : (QC_RS_IDLE_DUP ? pos_of(l - ZL) : pos_of(0));
    const bool store = QC_RS_IDLE_DUP ? true : live;
    // byte addresses of this lane's slot for a = 0 .. NA-1 (check side) and b = 0 .. Q-1 (variable side)
    int aC[NA], aV[Q];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        int p = zc + Q * a;
        p -= (p >= Z) ? Z : 0;
        aC[a] = 4 * (h * Z + p);
    }
#pragma unroll
    for (int b = 0; b < Q; ++b) {
        int p = zc - b;
        p += (p < 0) ? Z : 0;
        aV[b] = 4 * (h * Z + p);
    }
    // slot of edge (r, t) seen from the check side / the variable side (compile-time rotation, runtime base)
    auto cref = [&](auto rr, auto tt) __attribute__((always_inline)) -> float& {
        constexpr int r = decltype(rr)::value, t = decltype(tt)::value, s = C::SHR[r][t];
        int a = aC[s / Q];
        if constexpr (QC_RS_ADDR_OPAQUE) asm volatile("" : "+v"(a));  // one address VGPR per value of a
        return *reinterpret_cast<float*>(Xb + a + rs_rot_index<C>(r, t) * CROW);
    };
    auto vref = [&](auto rr, auto tt) __attribute__((always_inline)) -> float& {
        constexpr int r = decltype(rr)::value, t = decltype(tt)::value, s = C::SHR[r][t];
        int a = aV[s % Q];
        if constexpr (QC_RS_ADDR_OPAQUE) asm volatile("" : "+v"(a));
        return *reinterpret_cast<float*>(Xb + a + rs_rot_index<C>(r, t) * CROW);
    };
    // L = -llr (bp.py:47) of this lane's variable in block column j: in VGPRs, or re-read at every use (L2)
    const bool lval = QC_RS_IDLE_DUP ? cw < B : valid;  // shadow lanes load their partner's L
    const float* const lp = llr + (lval ? cw * N : 0);
    float Lreg[QC_RS_L == 0 ? NB : 1];
    auto Lload = [&](int j, bool opaque) __attribute__((always_inline)) {
        int z = zc;
        if (opaque) asm volatile("" : "+v"(z));
        int t = z + C::PHI[j];
        t -= (t >= Z) ? Z : 0;
        return lval ? -lp[j * Z + t] : 0.0f;
    };
    if constexpr (QC_RS_L == 0) {
#pragma unroll
        for (int j = 0; j < NB; ++j) Lreg[j] = Lload(j, false);
    }
    auto Lr_at = [&](int j) __attribute__((always_inline)) {
        if constexpr (QC_RS_L == 0) return Lreg[j];
        else return Lload(j, true);
    };
    float m0[N0 > 0 ? N0 : 1];  // messages of the rotation-0 circulants (both frames agree)
#pragma unroll
    for (int e = 0; e < N0; ++e) m0[e] = 0.0f;
    if (live) {  // c2v = 0 before the first iteration (bp.py:46: x = 0); each lane zeroes its check slots
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            static_for<0, C::DEG[decltype(rr)::value]>([&](auto tt) __attribute__((always_inline)) {
                if constexpr (C::SHR[decltype(rr)::value][decltype(tt)::value] != 0) cref(rr, tt) = 0.0f;
            });
        });
    }
    __syncthreads();  // every check slot zeroed
    const float cmax2 = sp_cmax2(clamp);  // check outputs in log2 units (common.h)
    // column j's messages in ascending row order: (row, slot) of its k-th edge
    auto col_rt = [](int j, int kk) constexpr {
        int c = 0;
        for (int r = 0; r < C::MB; ++r)
            for (int t = 0; t < C::DEG[r]; ++t)
                if (C::COL[r][t] == j) {
                    if (c == kk) return r * 64 + t;
                    ++c;
                }
        return -1;
    };
    auto vload = [&](auto jj, auto kk) __attribute__((always_inline)) {
        constexpr int rt = col_rt(decltype(jj)::value, decltype(kk)::value), r = rt / 64, t = rt % 64;
        if constexpr (C::SHR[r][t] == 0) return m0[rs_zero_index<C>(r, t)];
        else return vref(std::integral_constant<int, r>{}, std::integral_constant<int, t>{});
    };
    auto zsum = [&](auto jj) __attribute__((always_inline)) {  // z = 0.5 * (L + ascending sum of c2v)
        constexpr int j = decltype(jj)::value;
        float x[col_deg<C>(j)];
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) { x[kk] = vload(jj, kk); });
        float Ssum = 0.0f;
        static_for<0, col_deg<C>(j)>([&](auto kk) __attribute__((always_inline)) { Ssum += x[kk]; });
        return sp_z(Lr_at(j), Ssum);
    };

    // QC_RS_MASK_IDLE: idle lanes (l >= ZL) sit the iteration loop out, EXEC-masked (they never store; every wave
    // keeps live lanes, so each still meets both barriers of every iteration)
    const bool loop_lane = !QC_RS_MASK_IDLE || live;
    constexpr bool FIX = PASS == 2;
    // the rule applies per codeword (common.h): this lane's codeword's bit of the unit's flag
    uint32_t fixm = 0x7fffffffu;
    if constexpr (FIX) fixm = ((qc_sp_zflag(zlist, B)[unit] >> h) & 1u) ? 0x7fffffffu : 0u;
    if (loop_lane)
    for (int it = 0; it < iters; ++it) {
        // VN phase (variable frame): every column's c2v -> v2c as signed a, written back in place
        if constexpr (QC_RS_PRIO == 1 || QC_RS_PRIO == 3) __builtin_amdgcn_s_setprio(1);
        if constexpr (QC_RS_PRIO == 2) __builtin_amdgcn_s_setprio(0);
        if constexpr (QC_RS_PRIO == 4) __builtin_amdgcn_s_setprio(3);
        constexpr int DV = rs_max_col_deg<C>();
        float xn[DV];  // QC_RS_VPF: the next column's messages, loaded one column ahead
        if constexpr (QC_RS_VPF) {
            static_for<0, col_deg<C>(0)>([&](auto kk) __attribute__((always_inline)) {
                xn[kk] = vload(std::integral_constant<int, 0>{}, kk);
            });
        }
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            constexpr int dj = col_deg<C>(j);
            float x[dj];
            static_for<0, dj>([&](auto kk) __attribute__((always_inline)) {
                if constexpr (QC_RS_VPF) x[kk] = xn[kk];
                else x[kk] = vload(jj, kk);
            });
            if constexpr (QC_RS_VPF && j + 1 < NB) {  // other slots than column j's: no hazard with its stores
                static_for<0, col_deg<C>(j + 1)>([&](auto kk) __attribute__((always_inline)) {
                    xn[kk] = vload(std::integral_constant<int, j + 1>{}, kk);
                });
            }
            const float Lj = Lr_at(j);
            vn_excl_sums<dj, QC_RS_SERIAL>(
                [&](auto kk) __attribute__((always_inline)) { return x[kk]; },
                [&](auto kk, float Ssum) __attribute__((always_inline)) {
                    x[kk] = vn_signed_a(sp_vn_arg(Lj, Ssum));  // the (D, S) form's VC output (common.h)
                    if constexpr (QC_RS_SERIAL > 0 && (decltype(kk)::value + 1) % QC_RS_SERIAL == 0)
                        SP_TIE("+v"(x[kk]));
                });
            static_for<0, dj>([&](auto kk) __attribute__((always_inline)) {
                constexpr int rt = col_rt(j, decltype(kk)::value), r = rt / 64, t = rt % 64;
                if constexpr (C::SHR[r][t] == 0) m0[rs_zero_index<C>(r, t)] = x[kk];
            });
            if (store) {
                static_for<0, dj>([&](auto kk) __attribute__((always_inline)) {
                    constexpr int rt = col_rt(j, decltype(kk)::value), r = rt / 64, t = rt % 64;
                    if constexpr (C::SHR[r][t] != 0)
                        vref(std::integral_constant<int, r>{}, std::integral_constant<int, t>{}) = x[kk];
                });
            }
        });
        if constexpr (!QC_RS_DIAG_NOBAR) __syncthreads();  // (QC_RS_DIAG_NOBAR: diagnostic builds only)
        // CN phase (check frame): every row's v2c -> c2v, written back in place
        if constexpr (QC_RS_PRIO == 1 || QC_RS_PRIO == 3 || QC_RS_PRIO == 4) __builtin_amdgcn_s_setprio(0);
        if constexpr (QC_RS_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        constexpr int KP = QC_RS_CPF > 0 ? QC_RS_CPF : 1;
        float gn[KP];  // QC_RS_CPF: the last KP edges of the next row, loaded one row ahead
        auto cpf = [&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value, d = C::DEG[r];
            static_for<0, (KP < d ? KP : d)>([&](auto uu) __attribute__((always_inline)) {
                constexpr int t = d - 1 - decltype(uu)::value;
                if constexpr (C::SHR[r][t] != 0) gn[decltype(uu)::value] = cref(rr, std::integral_constant<int, t>{});
            });
        };
        if constexpr (QC_RS_CPF > 0) cpf(std::integral_constant<int, 0>{});
        static_for<0, MB>([&](auto rr) __attribute__((always_inline)) {
            constexpr int r = decltype(rr)::value;
            constexpr int d = C::DEG[r];
            if constexpr (QC_RS_PRIO == 3) __builtin_amdgcn_s_setprio(1);
            float g[d];
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                if constexpr (C::SHR[r][t] == 0) g[t] = m0[rs_zero_index<C>(r, t)];
                else if constexpr (QC_RS_CPF > 0 && t >= d - KP) g[t] = gn[d - 1 - t];
                else g[t] = cref(rr, tt);
            });
            if constexpr (QC_RS_PRIO == 3) __builtin_amdgcn_s_setprio(0);
            if constexpr (QC_RS_CPF > 0 && r + 1 < MB) cpf(std::integral_constant<int, r + 1>{});
            cn_ds_row<d, QC_RS_SERIAL_ROW, QC_RS_ROW_LAG, QC_RS_DS_BLOCK, FIX>(g, cmax2, fixm);  // O(d) exclusive sets (common.h)
            static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                constexpr int t = decltype(tt)::value;
                if constexpr (C::SHR[r][t] == 0) m0[rs_zero_index<C>(r, t)] = g[t];
            });
            if (store) {
                static_for<0, d>([&](auto tt) __attribute__((always_inline)) {
                    if constexpr (C::SHR[r][decltype(tt)::value] != 0) cref(rr, tt) = g[decltype(tt)::value];
                });
            }
        });
        if constexpr (!QC_RS_DIAG_NOBAR) __syncthreads();  // (QC_RS_DIAG_NOBAR: diagnostic builds only)
    }
    // the output's lane coordinates recomputed after the loop — the lane id by v_mbcnt (the work-item id VGPR of
    // the launch is long gone), the slot wave k is scalar — instead of kept across it: the values set before the
    // loop and read after it went to scratch (round 4: 63 MB of scratch stores per launch, WRITE_SIZE 1.92x the
    // bits out)
    const int lane_e = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const int le = lane_e & 31, he = (lane_e >> 5) & 1;
    const int64_t cwe = (PASS == 2 ? unit : (int64_t)blockIdx.x) * 2 + he;
    if (le < ZL && cwe < B) {
        const int zce = pos_of(le);
        static_for<0, NB>([&](auto jj) __attribute__((always_inline)) {
            constexpr int j = decltype(jj)::value;
            const float zz = zsum(jj);
            int t = zce + C::PHI[j];
            t -= (t >= Z) ? Z : 0;
            const int64_t o = cwe * N + j * Z + t;
            if (bits) bits[o] = (uint8_t)Num<float>::bit(zz);
            if (soft) soft[o] = (flags & LDPC_F_SOFT_Z) ? zz : 1.0f - 1.0f / (1.0f + Num<float>::exp_(-zz));
        });
        if (k == 0 && le == 0 && iters_used) iters_used[cwe] = iters;
    }
}

template <class C, int PASS = 1>
__global__ __launch_bounds__(C::S * 64) __attribute__((amdgpu_waves_per_eu(QC_RS_WAVES_PER_SIMD)))
void k_qc_sp_rs(const float* __restrict__ llr, int64_t B, int iters, float clamp, int flags,
                uint8_t* __restrict__ bits, float* __restrict__ soft, int32_t* __restrict__ iters_used,
                uint32_t* __restrict__ zlist) {
    if constexpr (PASS == 2) {  // the listed units, walked by this grid's workgroups
        const uint32_t n = zlist[0];
        for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
            qc_sp_rs_unit<C, 2>(__builtin_amdgcn_readfirstlane(zlist[1 + i]), llr, B, iters, clamp, flags, bits, soft,
                                iters_used, zlist);
            __syncthreads();  // the unit's last LDS reads before the next unit's writes
        }
    } else {
        qc_sp_rs_unit<C, PASS>(0, llr, B, iters, clamp, flags, bits, soft, iters_used, zlist);
    }
}

}  // namespace ldpc
