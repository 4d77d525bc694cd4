// Test-only kernel library (tests/test_gpu_cn_blocks.py; built by ldpc-sims_amd/build.py build_test_kernels):
// the tanh-SP check-row routine cn_ds_row (ldpc-sims_amd/csrc/common.h) instantiated at block sizes on the
// shared-T boundary ((d - 1) % BLOCK == 0: the last block's T is the row's last edge alone), off it, and as one
// block, with and without the a == 1 rule (FIX).  One thread per row; the test compares every blocked form with
// the one-block form bit for bit.  Not part of the product library.
#include <hip/hip_runtime.h>

#include "common.h"

namespace {

template <int d, int BLOCK, bool FIX>
__global__ __launch_bounds__(64) void k_cn_rows(const float* __restrict__ in, float* __restrict__ out, int rows,
                                                float cmax2) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    float g[d];
#pragma unroll
    for (int t = 0; t < d; ++t) g[t] = in[(int64_t)r * d + t];
    ldpc::cn_ds_row<d, 1, 0, BLOCK, FIX>(g, cmax2);
#pragma unroll
    for (int t = 0; t < d; ++t) out[(int64_t)r * d + t] = g[t];
}

template <int d, int BLOCK>
hipError_t launch(const float* in, float* out, int rows, int fix, float cmax2) {
    const unsigned blocks = (unsigned)((rows + 63) / 64);
    if (fix) k_cn_rows<d, BLOCK, true><<<blocks, 64>>>(in, out, rows, cmax2);
    else k_cn_rows<d, BLOCK, false><<<blocks, 64>>>(in, out, rows, cmax2);
    return hipGetLastError();
}

}  // namespace

// the (d, BLOCK) pairs instantiated: one block (BLOCK = d) and blocked forms, (d - 1) % BLOCK == 0 marked *
//   d = 14: 13*, 14          d = 15: 7*, 5, 15          d = 20: 19*, 7, 10, 20
extern "C" int cnrows_supported(int d, int block) {
    switch (d) {
        case 14: return block == 13 || block == 14;
        case 15: return block == 7 || block == 5 || block == 15;
        case 20: return block == 19 || block == 7 || block == 10 || block == 20;
        default: return 0;
    }
}

// rows x d signed a-values (|g| in (0, 1]: a = exp(-|s|), the sign of s) in, the row's outputs out (host
// pointers); cmax2 = the output ceiling in log2 units.  0 = ok, -1 = (d, block) not instantiated, -2 = HIP error.
extern "C" int cnrows_run(const float* g_host, float* out_host, int rows, int d, int block, int fix, float cmax2) {
    if (!cnrows_supported(d, block) || rows <= 0) return -1;
    const size_t bytes = (size_t)rows * d * sizeof(float);
    float *in = nullptr, *out = nullptr;
    if (hipMalloc((void**)&in, bytes) != hipSuccess) return -2;
    if (hipMalloc((void**)&out, bytes) != hipSuccess) {
        (void)hipFree(in);
        return -2;
    }
    hipError_t e = hipMemcpy(in, g_host, bytes, hipMemcpyHostToDevice);
#define CNR(D, BL) \
    if (e == hipSuccess && d == D && block == BL) e = launch<D, BL>(in, out, rows, fix, cmax2);
    CNR(14, 13) CNR(14, 14) CNR(15, 7) CNR(15, 5) CNR(15, 15) CNR(20, 19) CNR(20, 7) CNR(20, 10) CNR(20, 20)
#undef CNR
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out_host, out, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(in);
    (void)hipFree(out);
    return e == hipSuccess ? 0 : -2;
}
