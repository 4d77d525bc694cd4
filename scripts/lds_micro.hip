// lds_micro.hip — what the LDS pipe of one MI355X CU sustains for the headline kernel's instruction mix.
// Every CU runs 16 waves (4 per SIMD, as k_qc_ms_ph) of one of these loops. Each wave stamps the shader clock
// (s_memtime) and the 100 MHz real-time counter (s_memrealtime) around its loop: the chip-wide span comes from
// the real-time stamps, the in-kernel clock from their ratio (MI355X_MICROARCH.md, DVFS item 6), so rates are
// per shader cycle per CU at whatever clock the box runs (after ~1 s of back-to-back warm-up launches):
//   bperm   : 8 independent ds_bpermute_b32 chains per iteration (lane rotations, as the kernel's)
//   read128 : 8 independent ds_read_b128 per iteration (the kernel's L rows)
//   valu    : 8 independent v_fma chains per iteration (the VALU issue calibration)
//   mix     : per iteration 8 ds_bpermute + V VALU (V = 59: the kernel's 647 VALU per 88 bpermute) —
//             the same ratio without the kernel's dependencies: what the pipes give when perfectly fed
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_micro scripts/lds_micro.hip   Run: ./lds_micro > out.json
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                               \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

enum { BPERM = 0, READ128 = 1, VALU = 2, MIX = 3, ROT_ADDTID = 4, ROT_WRITE = 5 };

template <int MODE, int NV>
__global__ __launch_bounds__(256, 4) void k_micro(float* __restrict__ out, unsigned long long* __restrict__ cyc,
                                                  int iters, float a, int active) {
    __shared__ __attribute__((aligned(16))) float lds[256 * 8 + 4 * 64];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 256 * 8; i += 256) lds[i] = (float)i;
    __syncthreads();
    float v[8];
    int addr[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = (float)(lane + i);
        addr[i] = ((lane + 3 * i + 1) & 63) * 4;
    }
    float w[8];  // VALU chains, independent of the LDS results
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = (float)(lane - i);
    using f4 = __attribute__((ext_vector_type(4))) float;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    const int wv = threadIdx.x >> 6;
    const int rowf = 256 * 4 + wv * 64;  // this wave's rotation row (floats), after the b128 area
    const unsigned rowbase = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(&lds[rowf]));  // wave-uniform: M0
    const unsigned wa = rowbase + 4u * (unsigned)lane;
    const int rb = threadIdx.x * 4;  // 16 B per lane, lane-contiguous: conflict-free
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
    const bool on = (lane & 31) < active;  // lanes per 32-lane half taking part (27: the headline's Z)
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == BPERM || MODE == MIX) {
            if (on) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    v[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(addr[i], __float_as_int(v[i])));
            }
        }
        if constexpr (MODE == ROT_ADDTID || MODE == ROT_WRITE) {
            // a lane rotation through this wave's 256-B LDS row: store every lane's value at its own slot, load
            // the slot of lane (z + rho): the same address a ds_bpermute takes.  A wave's LDS operations are
            // processed in order, so one row serves every rotation without a wait or a barrier.
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (MODE == ROT_ADDTID)
                    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tds_write_addtid_b32 %0" ::"v"(v[i]), "s"(rowbase) : "memory", "m0");
                else
                    asm volatile("ds_write_b32 %0, %1" ::"v"(wa), "v"(v[i]) : "memory");
                v[i] = lds[rowf + (addr[i] >> 2)];
            }
        }
        if constexpr (MODE == READ128) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                int r = (rb + 1024 * ((i + it) & 1)) & (256 * 8 - 4);
                asm volatile("" : "+v"(r));
                acc += *static_cast<const f4*>(__builtin_assume_aligned(&lds[r], 16));
            }
        }
        if constexpr (MODE == VALU || MODE == MIX) {  // plain v_fmac_f32 (asm: no packed-math pairing)
            constexpr int n = (MODE == VALU) ? 64 : NV;
#pragma unroll
            for (int k = 0; k < n; ++k) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(w[k & 7]) : "v"(a), "v"(w[(k + 1) & 7]));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = acc.x + acc.y + acc.z + acc.w;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i] + w[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0) {
        unsigned long long* c = cyc + 4 * (blockIdx.x * 4 + (threadIdx.x >> 6));
        c[0] = r0;
        c[1] = r1;
        c[2] = t1 - t0;
    }
}

template <int MODE, int NV>
static int run(const char* name, int cus, int iters, int per_iter_lds, int per_iter_valu, int active, bool last) {
    const int blocks = cus * 4;  // 4 workgroups of 4 waves per CU: 16 waves per CU
    const int waves = blocks * 4;
    float* out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    CHECK(hipMalloc(&cyc, (size_t)waves * 4 * 8));
    for (int w = 0; w < 20; ++w) k_micro<MODE, NV><<<blocks, 256>>>(out, cyc, iters, 1.0000001f, active);  // clocks settle
    k_micro<MODE, NV><<<blocks, 256>>>(out, cyc, iters, 1.0000001f, active);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> c((size_t)waves * 4);
    CHECK(hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long rmin = ~0ull, rmax = 0;
    std::vector<double> clk;
    for (int w = 0; w < waves; ++w) {
        const unsigned long long a = c[4 * w], b = c[4 * w + 1], t = c[4 * w + 2];
        rmin = a < rmin ? a : rmin;
        rmax = b > rmax ? b : rmax;
        if (b > a) clk.push_back((double)t / (double)(b - a) * 0.1);  // GHz: shader cycles per 10 ns tick
    }
    std::sort(clk.begin(), clk.end());
    const double ghz = clk[clk.size() / 2];
    const double span_s = (double)(rmax - rmin) * 1e-8;
    const double span_cyc = span_s * ghz * 1e9;
    // per CU: 16 waves x iters x per_iter instructions within the chip-wide span
    const double lds_per_cu = 16.0 * iters * per_iter_lds, valu_per_simd = 4.0 * iters * per_iter_valu;
    printf("  {\"loop\": \"%s\", \"active_lanes_per_32\": %d, \"span_ms\": %.3f, \"clock_ghz\": %.3f", name, active,
           span_s * 1e3, ghz);
    if (per_iter_lds) printf(", \"cu_cycles_per_lds_instr\": %.3f", span_cyc / lds_per_cu);
    if (per_iter_valu) printf(", \"simd_cycles_per_valu_instr\": %.3f", span_cyc / valu_per_simd);
    printf("}%s\n", last ? "" : ",");
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
    return 0;
}

int main() {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    const int cus = prop.multiProcessorCount;
    const int iters = 100000;
    printf("{\"device\": \"%s\", \"cus\": %d, \"waves_per_cu\": 16, \"results\": [\n", prop.gcnArchName, cus);
    if (run<VALU, 0>("v_fmac_f32 x64", cus, iters, 0, 64, 32, false)) return 1;
    if (run<BPERM, 0>("ds_bpermute_b32 x8", cus, iters, 8, 0, 32, false)) return 1;
    if (run<BPERM, 0>("ds_bpermute_b32 x8", cus, iters, 8, 0, 27, false)) return 1;
    if (run<READ128, 0>("ds_read_b128 x8", cus, iters, 8, 0, 32, false)) return 1;
    if (run<ROT_ADDTID, 0>("rotation = ds_write_addtid_b32 + ds_read_b32, x8", cus, iters, 8, 0, 32, false)) return 1;
    if (run<ROT_WRITE, 0>("rotation = ds_write_b32 + ds_read_b32, x8", cus, iters, 8, 0, 32, false)) return 1;
    if (run<MIX, 59>("ds_bpermute_b32 x8 + v_fmac_f32 x59 (the headline's ratio)", cus, iters, 8, 59, 27, false)) return 1;
    if (run<MIX, 30>("ds_bpermute_b32 x8 + v_fmac_f32 x30", cus, iters, 8, 30, 27, true)) return 1;
    printf("]}\n");
    return 0;
}
