// abi.hip — the extern "C" surface of libldpc_hip.so (declared in include/ldpc_abi.h).
//
// Owns graph handles (CSR on device, built once: replaces generate_masks + BeliefPropagation.__init__,
// bp/masking.py:12-147, bp/bp.py:20-39), the workspace, host<->device staging for host-pointer callers
// (the reference's per-batch H2D / D2H at ofdm_functions.py:156,161), and dispatch between the
// structure-specialised QC kernels (qc.hip) and the generic CSR kernels (generic.hip).
#include <stdarg.h>
#include <stdio.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "host_pipeline.h"

struct ldpc_graph {
    int m = 0, n = 0, E = 0, device = 0;
    int max_dc = 0, max_dv = 0;
    int32_t *d_row_ptr = nullptr, *d_col_idx = nullptr, *d_var_ptr = nullptr, *d_var_edges = nullptr;
    int32_t* d_wofs = nullptr;  // weighted BP: [n+1] offsets of the per-variable d x d weight blocks
    int64_t W = 0;
    const ldpc::QCSpec* qc = nullptr;
    ldpc::IRASpec* ira = nullptr;  // DVB-S2-structured IRA code (ira.hip), when not QC
    std::mutex mtx;  // guards the internal workspace
    void* ws = nullptr;
    size_t ws_bytes = 0;
    // ldpc_decode_bits_host's staging ring (allocated on first use, reused; guarded by pipe_mtx)
    std::mutex pipe_mtx;
    struct Pipe {
        int64_t chunk = 0;        // codewords per slot
        size_t ws_bytes = 0;      // decode workspace per slot
        float* h_llr[2] = {};     // pinned host: float32 llr of one chunk
        uint8_t* h_bits[2] = {};  // pinned host: hard bits of one chunk
        float* d_llr[2] = {};
        uint8_t* d_bits[2] = {};
        void* d_ws[2] = {};
        hipStream_t st[2] = {};
        hipEvent_t done[2] = {};
    } pipe;
};

namespace ldpc {

static thread_local std::string g_err;

int set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

__global__ void k_fill_i32(int32_t* p, int64_t count, int32_t value) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) p[i] = value;
}

int fill_i32(int32_t* p, int64_t count, int32_t value, hipStream_t st) {
    if (count <= 0) return LDPC_OK;
    k_fill_i32<<<(unsigned)((count + 255) / 256), 256, 0, st>>>(p, count, value);
    return LDPC_OK;
}

// Error counting (evaluate_quantized.py:139-141): one wave per codeword, wave-reduced, one atomic per wave.
__global__ __launch_bounds__(256) void k_count_errors(const uint8_t* __restrict__ bits, const uint8_t* __restrict__ ref,
                                                      int64_t B, int n, int info, unsigned long long* counts) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    unsigned long long be = 0, blk = 0;
    for (int64_t b = wave; b < B; b += nwaves) {
        int e_info = 0, e_all = 0;
        for (int v = lane; v < n; v += 64) {
            const int r = ref ? ref[b * n + v] : 0;
            const int d = (bits[b * n + v] != r);
            e_all |= d;
            e_info += (v < info) ? d : 0;
        }
        for (int o = 32; o > 0; o >>= 1) {
            e_info += __shfl_xor(e_info, o);
            e_all |= __shfl_xor(e_all, o);
        }
        be += (unsigned long long)e_info;
        blk += (unsigned long long)e_all;
    }
    if (lane == 0) {
        if (be) atomicAdd(&counts[0], be);
        if (blk) atomicAdd(&counts[1], blk);
    }
}

__global__ void k_add_count(unsigned long long* counts, unsigned long long B) { atomicAdd(&counts[2], B); }

// On-device BPSK/AWGN.  Element gi = (b0+b)*n + v draws normal gi from
// Philox(counter = gi/4, key = seed) + Box-Muller, so a shard's LLRs do not depend on the shard size.
__global__ __launch_bounds__(256) void k_awgn(const uint8_t* __restrict__ cw, float* __restrict__ llr, int64_t B, int n,
                                              float sigma, uint64_t seed, int64_t b0) {
    const int64_t first = b0 * n, last = (b0 + B) * n;  // global element range
    const int64_t q = first / 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q * 4 >= last) return;
    uint32_t r[4];
    Philox::gen((uint64_t)q, seed, r);
    float z[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const float u1 = ((float)r[2 * h] + 1.0f) * 2.3283064365386963e-10f;  // (0, 1]
        const float u2 = (float)r[2 * h + 1] * 2.3283064365386963e-10f;       // [0, 1)
        const float rad = sqrtf(-2.0f * logf(u1));
        float s, c;
        sincospif(2.0f * u2, &s, &c);
        z[2 * h] = rad * c;
        z[2 * h + 1] = rad * s;
    }
    const float k = -2.0f / (sigma * sigma);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t gi = q * 4 + j;
        if (gi < first || gi >= last) continue;
        const int64_t li = gi - first;
        const float s = cw ? (1.0f - 2.0f * (float)cw[li]) : 1.0f;
        llr[li] = k * (s + sigma * z[j]);
    }
}

__global__ __launch_bounds__(256) void k_random_bits(uint8_t* __restrict__ out, int64_t B, int k, uint64_t seed,
                                                     int64_t b0) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * k) return;
    uint32_t r[4];
    Philox::gen((uint64_t)(b0 * k + i), seed ^ 0x9E3779B97F4A7C15ull, r);
    out[i] = (uint8_t)(r[0] & 1u);
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static bool params_valid(const ldpc_params* p) {
    if (!p) return false;
    if (p->iters < 0 || p->iters > 100000) return false;
    if (p->algo < LDPC_ALGO_TANH_SP || p->algo > LDPC_ALGO_QMIN_SUM) return false;
    if (!(p->clamp > 0.0f)) return false;
    if (p->algo == LDPC_ALGO_MIN_SUM && !(p->alpha > 0.0f)) return false;
    if (p->algo == LDPC_ALGO_QMIN_SUM && (p->qmax < 1 || p->qmax > 127 || p->app_max < p->qmax ||
                                          p->app_max > 32767 || !(p->qstep > 0.0f)))
        return false;
    // integer offset min-sum: no normalisation, a whole non-negative offset (the kernels and the oracle's
    // qms work in small integers; a fractional beta would silently truncate)
    if (p->algo == LDPC_ALGO_QMIN_SUM && (p->alpha != 1.0f || !(p->beta >= 0.0f) || p->beta != floorf(p->beta) ||
                                          p->beta > (float)p->qmax))
        return false;
    return true;
}

static GenericArgs gargs(const ldpc_graph* g) {
    return GenericArgs{g->d_row_ptr, g->d_col_idx, g->d_var_ptr, g->d_var_edges, g->m, g->n, g->E, g->max_dc, g->max_dv,
                       g->d_wofs, g->W};
}

static bool use_qc(const ldpc_graph* g, const ldpc_params* p) {
    return g->qc && !(p->flags & LDPC_F_FORCE_GENERIC) && qc_supports(g->qc, *p);
}

static bool use_ira(const ldpc_graph* g, const ldpc_params* p) {
    return g->ira && !(p->flags & LDPC_F_FORCE_GENERIC) && ira_supports(g->ira, *p);
}

static size_t elem_size(const ldpc_params* p) { return (p->flags & LDPC_F_F64) ? 8 : 4; }

// Workspace = kernel scratch followed (host-pointer callers only) by staging for llr/bits/soft/used.
static size_t kernel_ws(const ldpc_graph* g, int64_t B, const ldpc_params* p) {
    if (use_qc(g, p)) return align256(qc_workspace(g->qc, B, *p));
    if (use_ira(g, p)) return align256(ira_workspace(g->ira, B, *p));
    return align256(generic_workspace(gargs(g), B, *p));
}
static size_t staging_ws(const ldpc_graph* g, int64_t B, const ldpc_params* p) {
    if (p->flags & LDPC_F_DEVICE_PTRS) return 0;
    const size_t es = elem_size(p);
    return align256((size_t)B * g->n * es) + align256((size_t)B * g->n) + align256((size_t)B * g->n * es) +
           align256((size_t)B * 4);
}

static int build_graph(ldpc_graph* g, int m, int n, const std::vector<int32_t>& row_ptr,
                       const std::vector<int32_t>& col_idx) {
    const int E = (int)col_idx.size();
    g->m = m;
    g->n = n;
    g->E = E;
    std::vector<int32_t> var_ptr(n + 1, 0), var_edges(E);
    for (int e = 0; e < E; ++e) var_ptr[col_idx[e] + 1]++;
    for (int v = 0; v < n; ++v) var_ptr[v + 1] += var_ptr[v];
    std::vector<int32_t> fill(var_ptr.begin(), var_ptr.end() - 1);
    for (int c = 0; c < m; ++c)  // ascending check within a column (masking.py:91-95)
        for (int e = row_ptr[c]; e < row_ptr[c + 1]; ++e) var_edges[fill[col_idx[e]]++] = e;
    g->max_dc = 0;
    for (int c = 0; c < m; ++c) g->max_dc = std::max(g->max_dc, row_ptr[c + 1] - row_ptr[c]);
    g->max_dv = 0;
    for (int v = 0; v < n; ++v) g->max_dv = std::max(g->max_dv, var_ptr[v + 1] - var_ptr[v]);
    std::vector<int32_t> wofs(n + 1, 0);
    int64_t W = 0;
    for (int v = 0; v < n; ++v) {
        const int64_t d = var_ptr[v + 1] - var_ptr[v];
        W += d * d;
        if (W > INT32_MAX) return set_error(LDPC_EUNSUPPORTED, "weight layout exceeds int32 offsets");
        wofs[v + 1] = (int32_t)W;
    }
    g->W = W;
    DeviceGuard dg(g->device);
    auto up = [](int32_t** d, const std::vector<int32_t>& h) -> hipError_t {
        hipError_t e = hipMalloc((void**)d, std::max<size_t>(4, h.size() * 4));
        if (e != hipSuccess) return e;
        return hipMemcpy(*d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    };
    hipError_t e;
    if ((e = up(&g->d_row_ptr, row_ptr)) != hipSuccess || (e = up(&g->d_col_idx, col_idx)) != hipSuccess ||
        (e = up(&g->d_var_ptr, var_ptr)) != hipSuccess ||
        (e = up(&g->d_var_edges, var_edges)) != hipSuccess || (e = up(&g->d_wofs, wofs)) != hipSuccess)
        return set_error(e == hipErrorOutOfMemory ? LDPC_ENOMEM : LDPC_EHIP, "graph upload: %s", hipGetErrorString(e));
    return LDPC_OK;
}

// Recognise H as the lifting of a base matrix with a compiled QC kernel.
static const QCSpec* detect_qc(int m, int n, const std::vector<int32_t>& row_ptr, const std::vector<int32_t>& col_idx) {
    static const int zs[] = {27, 54, 81, 96, 360};
    for (int z : zs) {
        if (m % z || n % z) continue;
        const int mb = m / z, nb = n / z;
        std::vector<int32_t> sh((size_t)mb * nb, -1);
        bool ok = true;
        // row r*z+0 of each block row defines the shifts; verify every row of every block.
        for (int r = 0; r < mb && ok; ++r)
            for (int e = row_ptr[r * z]; e < row_ptr[r * z + 1]; ++e) {
                const int j = col_idx[e] / z;
                sh[(size_t)r * nb + j] = col_idx[e] % z;
            }
        for (int r = 0; r < mb && ok; ++r)
            for (int i = 0; i < z && ok; ++i) {
                const int c = r * z + i;
                int cnt = 0;
                for (int j = 0; j < nb; ++j) cnt += sh[(size_t)r * nb + j] >= 0;
                if (row_ptr[c + 1] - row_ptr[c] != cnt) { ok = false; break; }
                int e = row_ptr[c];
                for (int j = 0; j < nb; ++j) {
                    const int s = sh[(size_t)r * nb + j];
                    if (s < 0) continue;
                    if (col_idx[e++] != j * z + (i + s) % z) { ok = false; break; }
                }
            }
        if (!ok) continue;
        if (const QCSpec* spec = qc_lookup(mb, nb, z, sh.data())) return spec;
    }
    return nullptr;
}

// ---- staging ring of ldpc_decode_bits_host --------------------------------------------------------
static void pipe_free(ldpc_graph* g) {
    auto& P = g->pipe;
    for (int i = 0; i < 2; ++i) {
        if (P.done[i]) (void)hipEventDestroy(P.done[i]);
        if (P.st[i]) (void)hipStreamDestroy(P.st[i]);
        if (P.h_llr[i]) (void)hipHostFree(P.h_llr[i]);
        if (P.h_bits[i]) (void)hipHostFree(P.h_bits[i]);
        if (P.d_llr[i]) (void)hipFree(P.d_llr[i]);
        if (P.d_bits[i]) (void)hipFree(P.d_bits[i]);
        if (P.d_ws[i]) (void)hipFree(P.d_ws[i]);
    }
    P = ldpc_graph::Pipe{};
}

static int pipe_alloc(ldpc_graph* g, int64_t chunk, size_t ws_bytes) {
    auto& P = g->pipe;
    if (P.chunk >= chunk && P.ws_bytes >= ws_bytes) return LDPC_OK;
    pipe_free(g);
    const size_t nl = (size_t)chunk * g->n;
    for (int i = 0; i < 2; ++i) {
        hipError_t e = hipHostMalloc((void**)&P.h_llr[i], nl * 4, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void**)&P.h_bits[i], nl, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc((void**)&P.d_llr[i], nl * 4);
        if (e == hipSuccess) e = hipMalloc((void**)&P.d_bits[i], nl);
        if (e == hipSuccess) e = hipMalloc(&P.d_ws[i], ws_bytes);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&P.st[i], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&P.done[i], hipEventDisableTiming);
        if (e != hipSuccess) {
            pipe_free(g);
            return set_error(LDPC_ENOMEM, "decode_bits staging (%lld codewords): %s", (long long)chunk, hipGetErrorString(e));
        }
    }
    P.chunk = chunk;
    P.ws_bytes = ws_bytes;
    return LDPC_OK;
}

}  // namespace ldpc

using namespace ldpc;

extern "C" {

const char* ldpc_last_error(void) { return g_err.c_str(); }

const char* ldpc_version(void) { return "ldpc-mi355x 0.2 (gfx950)"; }

int ldpc_abi_version(void) { return LDPC_ABI_VERSION; }

int ldpc_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

int ldpc_graph_create(int32_t m, int32_t n, int32_t nnz, const int32_t* row_ptr, const int32_t* col_idx,
                      int32_t device, ldpc_graph** out) {
    if (!out || !row_ptr || !col_idx || m <= 0 || n <= 0 || nnz <= 0) return set_error(LDPC_EINVAL, "bad graph arguments");
    *out = nullptr;
    std::vector<int32_t> rp(row_ptr, row_ptr + m + 1), ci(col_idx, col_idx + nnz);
    if (rp[0] != 0 || rp[m] != nnz) return set_error(LDPC_EINVAL, "row_ptr must start at 0 and end at nnz");
    for (int c = 0; c < m; ++c) {
        if (rp[c + 1] < rp[c]) return set_error(LDPC_EINVAL, "row_ptr not monotone at row %d", c);
        for (int e = rp[c]; e < rp[c + 1]; ++e) {
            if (ci[e] < 0 || ci[e] >= n) return set_error(LDPC_EINVAL, "col_idx out of range at edge %d", e);
            if (e > rp[c] && ci[e] <= ci[e - 1]) return set_error(LDPC_EINVAL, "columns of row %d not strictly ascending", c);
        }
    }
    int ndev = ldpc_device_count();
    if (device < 0 || device >= ndev) return set_error(LDPC_EINVAL, "device %d out of range (%d visible)", device, ndev);
    ldpc_graph* g = new ldpc_graph();
    g->device = device;
    int rc = build_graph(g, m, n, rp, ci);
    if (rc != LDPC_OK) {
        ldpc_graph_destroy(g);
        return rc;
    }
    g->qc = detect_qc(m, n, rp, ci);
    if (!g->qc) g->ira = ira_detect(m, n, rp.data(), ci.data(), device);
    *out = g;
    return LDPC_OK;
}

int ldpc_graph_create_qc(int32_t mb, int32_t nb, int32_t z, const int32_t* shifts, int32_t device, ldpc_graph** out) {
    if (!out || !shifts || mb <= 0 || nb <= 0 || z <= 0) return set_error(LDPC_EINVAL, "bad QC arguments");
    std::vector<int32_t> rp(1, 0), ci;
    for (int r = 0; r < mb; ++r)
        for (int i = 0; i < z; ++i) {
            for (int j = 0; j < nb; ++j) {
                const int s = shifts[(size_t)r * nb + j];
                if (s >= z) return set_error(LDPC_EINVAL, "shift %d >= z at (%d,%d)", s, r, j);
                if (s >= 0) ci.push_back(j * z + (i + s) % z);
            }
            rp.push_back((int32_t)ci.size());
        }
    if (ci.empty()) return set_error(LDPC_EINVAL, "empty base matrix");
    return ldpc_graph_create(mb * z, nb * z, (int32_t)ci.size(), rp.data(), ci.data(), device, out);
}

int ldpc_graph_destroy(ldpc_graph* g) {
    if (!g) return LDPC_OK;
    DeviceGuard dg(g->device);
    (void)hipFree(g->d_row_ptr);
    (void)hipFree(g->d_col_idx);
    (void)hipFree(g->d_var_ptr);
    (void)hipFree(g->d_var_edges);
    (void)hipFree(g->d_wofs);
    ira_free(g->ira);
    if (g->ws) (void)hipFree(g->ws);
    pipe_free(g);
    delete g;
    return LDPC_OK;
}

int ldpc_graph_info(const ldpc_graph* g, int32_t* m, int32_t* n, int32_t* nnz, int32_t* z) {
    if (!g) return set_error(LDPC_EINVAL, "null graph");
    if (m) *m = g->m;
    if (n) *n = g->n;
    if (nnz) *nnz = g->E;
    if (z) *z = g->qc ? qc_z(g->qc) : 0;
    return LDPC_OK;
}

const char* ldpc_kernel_path(const ldpc_graph* g, const ldpc_params* p) {
    static thread_local std::string path;
    if (!g || !params_valid(p)) {
        set_error(LDPC_EINVAL, "bad kernel_path query");
        return nullptr;
    }
    if (use_qc(g, p)) path = "qc-z" + std::to_string(qc_z(g->qc));
    else if (use_ira(g, p)) path = "ira-z360";
    else path = "generic-csr";
    return path.c_str();
}

int ldpc_workspace_size(const ldpc_graph* g, int64_t B, const ldpc_params* p, size_t* bytes) {
    if (!g || !bytes || B < 0 || !params_valid(p)) return set_error(LDPC_EINVAL, "bad workspace query");
    *bytes = kernel_ws(g, B, p) + staging_ws(g, B, p);
    return LDPC_OK;
}

static int decode_impl(const ldpc_graph* gc, const void* llr, int64_t B, const ldpc_params* p, uint8_t* bits_out,
                       void* soft_out, int32_t* iters_used, void* workspace, size_t workspace_bytes, void* stream,
                       const BPWeights* w) {
    ldpc_graph* g = const_cast<ldpc_graph*>(gc);
    if (!g) return set_error(LDPC_EINVAL, "null graph");
    if (!params_valid(p)) return set_error(LDPC_EINVAL, "invalid ldpc_params");
    if (B < 0 || (B > 0 && !llr)) return set_error(LDPC_EINVAL, "llr is null or B < 0");
    if (B == 0) return LDPC_OK;
    if (p->algo == LDPC_ALGO_QMIN_SUM && !use_qc(g, p))
        return set_error(LDPC_EUNSUPPORTED, "quantized min-sum needs a QC-specialised graph");
    DeviceGuard dg(g->device);
    hipStream_t st = (hipStream_t)stream;
    const size_t need_k = kernel_ws(g, B, p), need_s = staging_ws(g, B, p);
    std::unique_lock<std::mutex> lock;
    char* ws = (char*)workspace;
    if (ws) {
        if (workspace_bytes < need_k + need_s)
            return set_error(LDPC_ENOMEM, "workspace %zu bytes < required %zu", workspace_bytes, need_k + need_s);
    } else {
        lock = std::unique_lock<std::mutex>(g->mtx);
        if (g->ws_bytes < need_k + need_s) {
            if (g->ws) (void)hipFree(g->ws);
            g->ws = nullptr;
            g->ws_bytes = 0;
            hipError_t e = hipMalloc(&g->ws, need_k + need_s);
            if (e != hipSuccess) return set_error(LDPC_ENOMEM, "workspace alloc %zu: %s", need_k + need_s, hipGetErrorString(e));
            g->ws_bytes = need_k + need_s;
        }
        ws = (char*)g->ws;
    }
    const bool dev = (p->flags & LDPC_F_DEVICE_PTRS) != 0;
    const size_t es = elem_size(p);
    const void* llr_d = llr;
    uint8_t* bits_d = bits_out;
    void* soft_d = soft_out;
    int32_t* used_d = iters_used;
    hipError_t e;
    if (!dev) {
        char* s = ws + need_k;
        void* llr_s = s;
        s += align256((size_t)B * g->n * es);
        bits_d = bits_out ? (uint8_t*)s : nullptr;
        s += align256((size_t)B * g->n);
        soft_d = soft_out ? (void*)s : nullptr;
        s += align256((size_t)B * g->n * es);
        used_d = iters_used ? (int32_t*)s : nullptr;
        if ((e = hipMemcpyAsync(llr_s, llr, (size_t)B * g->n * es, hipMemcpyHostToDevice, st)) != hipSuccess)
            return set_error(LDPC_EHIP, "llr H2D: %s", hipGetErrorString(e));
        llr_d = llr_s;
    }
    int rc;
    if (use_qc(g, p)) {
        rc = qc_decode(g->qc, llr_d, B, *p, bits_d, soft_d, used_d, ws, st);
    } else if (use_ira(g, p) && !w) {
        rc = ira_decode(g->ira, (const float*)llr_d, B, *p, bits_d, (float*)soft_d, used_d, ws, st);
    } else {
        rc = generic_decode(gargs(g), llr_d, B, *p, bits_d, soft_d, used_d, ws, st, w);
    }
    if (rc != LDPC_OK) return rc;
    if (!dev) {
        if (bits_out && (e = hipMemcpyAsync(bits_out, bits_d, (size_t)B * g->n, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return set_error(LDPC_EHIP, "bits D2H: %s", hipGetErrorString(e));
        if (soft_out && (e = hipMemcpyAsync(soft_out, soft_d, (size_t)B * g->n * es, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return set_error(LDPC_EHIP, "soft D2H: %s", hipGetErrorString(e));
        if (iters_used && (e = hipMemcpyAsync(iters_used, used_d, (size_t)B * 4, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return set_error(LDPC_EHIP, "iters D2H: %s", hipGetErrorString(e));
    }
    if (!dev || !workspace) {
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return set_error(LDPC_EHIP, "decode: %s", hipGetErrorString(e));
    }
    return LDPC_OK;
}

int ldpc_decode_ex(const ldpc_graph* g, const void* llr, int64_t B, const ldpc_params* p, uint8_t* bits_out,
                   void* soft_out, int32_t* iters_used, void* workspace, size_t workspace_bytes, void* stream) {
    return decode_impl(g, llr, B, p, bits_out, soft_out, iters_used, workspace, workspace_bytes, stream, nullptr);
}

int ldpc_weights_layout(const ldpc_graph* g, int64_t* vn_per_iter, int64_t* fin_len) {
    if (!g) return set_error(LDPC_EINVAL, "null graph");
    if (vn_per_iter) *vn_per_iter = g->W;
    if (fin_len) *fin_len = g->E;
    return LDPC_OK;
}

int ldpc_decode_weighted(const ldpc_graph* g, const void* llr, int64_t B, const ldpc_params* p,
                         const ldpc_bp_weights* w, uint8_t* bits_out, void* soft_out, int32_t* iters_used,
                         void* workspace, size_t workspace_bytes, void* stream) {
    if (!p || !params_valid(p)) return set_error(LDPC_EINVAL, "invalid ldpc_params");
    if (p->algo != LDPC_ALGO_TANH_SP || (p->flags & LDPC_F_EARLY_STOP))
        return set_error(LDPC_EUNSUPPORTED, "weighted BP is tanh sum-product without early stop");
    ldpc_params q = *p;
    q.flags |= LDPC_F_FORCE_GENERIC;
    const BPWeights bw{w ? w->vn : nullptr, w ? w->llr : nullptr, w ? w->fin : nullptr, w ? w->fin_llr : nullptr};
    return decode_impl(g, llr, B, &q, bits_out, soft_out, iters_used, workspace, workspace_bytes, stream, &bw);
}

int ldpc_decode_x0(const ldpc_graph* g, const void* llr, int64_t B, const ldpc_params* p, const ldpc_bp_weights* w,
                   const void* x0, uint8_t* bits_out, void* soft_out, int32_t* iters_used, void* workspace,
                   size_t workspace_bytes, void* stream) {
    if (!p || !params_valid(p)) return set_error(LDPC_EINVAL, "invalid ldpc_params");
    if (p->algo != LDPC_ALGO_TANH_SP || (p->flags & LDPC_F_EARLY_STOP))
        return set_error(LDPC_EUNSUPPORTED, "initial messages: tanh sum-product without early stop");
    if (x0 && !(p->flags & LDPC_F_DEVICE_PTRS)) return set_error(LDPC_EINVAL, "x0 needs LDPC_F_DEVICE_PTRS");
    ldpc_params q = *p;
    q.flags |= LDPC_F_FORCE_GENERIC;
    BPWeights bw{w ? w->vn : nullptr, w ? w->llr : nullptr, w ? w->fin : nullptr, w ? w->fin_llr : nullptr};
    bw.c2v0 = x0;
    return decode_impl(g, llr, B, &q, bits_out, soft_out, iters_used, workspace, workspace_bytes, stream, &bw);
}

int ldpc_decode(const ldpc_graph* g, const float* llr, int64_t B, int32_t iters, float clamp, int32_t algo,
                int32_t flags, uint8_t* bits_out, float* soft_out, int32_t* iters_used, void* stream) {
    ldpc_params p{};
    p.iters = iters;
    p.algo = algo;
    p.flags = flags & ~LDPC_F_F64;
    p.clamp = clamp;
    p.alpha = 1.0f;
    p.beta = 0.0f;
    p.qmax = 15;
    p.app_max = 127;
    p.qstep = 1.0f;
    return ldpc_decode_ex(g, llr, B, &p, bits_out, soft_out, iters_used, nullptr, 0, stream);
}

int ldpc_decode_bits_host(const ldpc_graph* gc, const double* llr, int64_t rows, const ldpc_params* p, double* out,
                          int64_t chunk, int32_t threads) {
    ldpc_graph* g = const_cast<ldpc_graph*>(gc);
    if (!g || !p || rows < 0 || (rows > 0 && (!llr || !out))) return set_error(LDPC_EINVAL, "bad decode_bits arguments");
    if (!params_valid(p)) return set_error(LDPC_EINVAL, "invalid ldpc_params");
    if (p->flags & (LDPC_F_F64 | LDPC_F_DEVICE_PTRS | LDPC_F_SOFT_Z))
        return set_error(LDPC_EINVAL, "decode_bits_host: float32 arithmetic on host buffers, bits only");
    if (rows == 0) return LDPC_OK;
    const int n = g->n;
    if (chunk <= 0) chunk = std::max<int64_t>(256, ((int64_t)16 << 20) / ((int64_t)n * 4) / 256 * 256);  // ~16 MB of f32
    chunk = std::min(chunk, rows);
    if (threads <= 0) threads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    ldpc_params q = *p;
    q.flags |= LDPC_F_DEVICE_PTRS;
    DeviceGuard dg(g->device);
    std::lock_guard<std::mutex> lock(g->pipe_mtx);
    int rc = pipe_alloc(g, chunk, std::max<size_t>(256, kernel_ws(g, chunk, &q)));
    if (rc != LDPC_OK) return rc;
    auto& P = g->pipe;
    hipError_t e;
    for (int i = 0; i < 2; ++i)  // a previous call that failed midway may still have copies in flight
        if ((e = hipStreamSynchronize(P.st[i])) != hipSuccess)
            return set_error(LDPC_EHIP, "decode_bits: %s", hipGetErrorString(e));
    // the engine of the two-slot staging pipeline (host_pipeline.h): H2D, decode, D2H and a completion
    // event per slot on that slot's stream
    struct HipEngine {
        ldpc_graph* g;
        ldpc_graph::Pipe& P;
        const ldpc_params* q;
        int n;
        float* h_llr(int s) { return P.h_llr[s]; }
        const uint8_t* h_bits(int s) { return P.h_bits[s]; }
        int submit(int s, int64_t nr) {
            hipError_t e;
            hipStream_t st = P.st[s];
            if ((e = hipMemcpyAsync(P.d_llr[s], P.h_llr[s], (size_t)nr * n * 4, hipMemcpyHostToDevice, st)) != hipSuccess)
                return set_error(LDPC_EHIP, "decode_bits H2D: %s", hipGetErrorString(e));
            const int rc = decode_impl(g, P.d_llr[s], nr, q, P.d_bits[s], nullptr, nullptr, P.d_ws[s], P.ws_bytes, st,
                                       nullptr);
            if (rc != LDPC_OK) return rc;
            if ((e = hipMemcpyAsync(P.h_bits[s], P.d_bits[s], (size_t)nr * n, hipMemcpyDeviceToHost, st)) != hipSuccess)
                return set_error(LDPC_EHIP, "decode_bits D2H: %s", hipGetErrorString(e));
            if ((e = hipEventRecord(P.done[s], st)) != hipSuccess)
                return set_error(LDPC_EHIP, "decode_bits event: %s", hipGetErrorString(e));
            return LDPC_OK;
        }
        int wait(int s) {
            const hipError_t e = hipEventSynchronize(P.done[s]);
            return e == hipSuccess ? LDPC_OK : set_error(LDPC_EHIP, "decode_bits: %s", hipGetErrorString(e));
        }
    } eng{g, P, &q, n};
    return staging_pipeline(eng, llr, rows, n, chunk, threads, out);
}

int ldpc_count_errors(const uint8_t* bits, const uint8_t* ref, int64_t B, int32_t n, int32_t info_bits, int64_t* counts,
                      void* stream) {
    if (!bits || !counts || B < 0 || n <= 0 || info_bits < 0 || info_bits > n)
        return set_error(LDPC_EINVAL, "bad count_errors arguments");
    if (B == 0) return LDPC_OK;
    hipStream_t st = (hipStream_t)stream;
    const int64_t blocks = std::min<int64_t>((B + 3) / 4, 4096);
    k_count_errors<<<(unsigned)blocks, 256, 0, st>>>(bits, ref, B, n, info_bits, (unsigned long long*)counts);
    k_add_count<<<1, 1, 0, st>>>((unsigned long long*)counts, (unsigned long long)B);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "count_errors: %s", hipGetErrorString(e));
    return LDPC_OK;
}

int ldpc_awgn_llr(const uint8_t* codeword, float* llr, int64_t B, int32_t n, float sigma, uint64_t seed, int64_t b0,
                  void* stream) {
    if (!llr || B < 0 || n <= 0 || !(sigma > 0.0f) || b0 < 0) return set_error(LDPC_EINVAL, "bad awgn arguments");
    if (B == 0) return LDPC_OK;
    const int64_t first = b0 * n, last = (b0 + B) * n;
    const int64_t quads = (last + 3) / 4 - first / 4;
    k_awgn<<<(unsigned)((quads + 255) / 256), 256, 0, (hipStream_t)stream>>>(codeword, llr, B, n, sigma, seed, b0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "awgn: %s", hipGetErrorString(e));
    return LDPC_OK;
}

int ldpc_random_bits(uint8_t* out, int64_t B, int32_t k, uint64_t seed, int64_t b0, void* stream) {
    if (!out || B < 0 || k <= 0 || b0 < 0) return set_error(LDPC_EINVAL, "bad random_bits arguments");
    if (B == 0) return LDPC_OK;
    k_random_bits<<<(unsigned)((B * k + 255) / 256), 256, 0, (hipStream_t)stream>>>(out, B, k, seed, b0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "random_bits: %s", hipGetErrorString(e));
    return LDPC_OK;
}

}  // extern "C"
