// generic.hip — entry points of the generic CSR decoder: workspace size, Infinity-Cache-sized chunking, and
// dispatch to the driver instantiations (kernels and drivers: generic_impl.h / generic_run.hip).
#include "generic_impl.h"

namespace ldpc {

size_t generic_workspace(const GenericArgs& g, int64_t B, const ldpc_params& p) {
    const size_t elem = (p.flags & LDPC_F_F64) ? 8 : 4;
    return layout(g, chunk_cw(g, B, p), elem, (p.flags & LDPC_F_EARLY_STOP) != 0).total;
}

// driver instantiations, one translation unit each (generic_run.hip, build.py)
#define LDPC_RUN_DECL(name) \
    int name(const GenericArgs& g, const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft, \
             int32_t* iters_used, char* ws, hipStream_t st, const BPWeights* w);
LDPC_RUN_DECL(generic_run_sp32)
LDPC_RUN_DECL(generic_run_sp32_es)
LDPC_RUN_DECL(generic_run_sp64)
LDPC_RUN_DECL(generic_run_sp64_es)
LDPC_RUN_DECL(generic_run_ms32)
LDPC_RUN_DECL(generic_run_ms32_es)
#undef LDPC_RUN_DECL

static int decode_chunk(const GenericArgs& g, const void* llr_dev, int64_t B, const ldpc_params& p, uint8_t* bits,
                        void* soft, int32_t* iters_used, char* ws, hipStream_t st, const BPWeights* w);

int generic_decode(const GenericArgs& g, const void* llr_dev, int64_t B, const ldpc_params& p, uint8_t* bits,
                   void* soft, int32_t* iters_used, char* ws, hipStream_t st, const BPWeights* w) {
    const size_t elem = (p.flags & LDPC_F_F64) ? 8 : 4;
    const int64_t bc = chunk_cw(g, B, p);
    for (int64_t o = 0; o < B; o += bc) {
        const int64_t b = (B - o < bc) ? B - o : bc;
        const int64_t vo = o * g.n;
        BPWeights wc{};
        if (w) {
            wc = *w;
            if (w->c2v0) wc.c2v0 = (const char*)w->c2v0 + o * (int64_t)g.E * (int64_t)elem;
        }
        const int rc = decode_chunk(g, (const char*)llr_dev + vo * elem, b, p, bits ? bits + vo : nullptr,
                                    soft ? (void*)((char*)soft + vo * elem) : nullptr, iters_used ? iters_used + o : nullptr,
                                    ws, st, w ? &wc : nullptr);
        if (rc != LDPC_OK) return rc;
    }
    return LDPC_OK;
}

static int decode_chunk(const GenericArgs& g, const void* llr_dev, int64_t B, const ldpc_params& p, uint8_t* bits,
                        void* soft, int32_t* iters_used, char* ws, hipStream_t st, const BPWeights* w) {
    const bool es = (p.flags & LDPC_F_EARLY_STOP) != 0;
    if (w && (p.algo != LDPC_ALGO_TANH_SP || es))
        return set_error(LDPC_EUNSUPPORTED, "weighted BP / initial messages: tanh sum-product without early stop");
    int rc;
    if (p.algo == LDPC_ALGO_TANH_SP) {
        if (p.flags & LDPC_F_F64) {
            const double* x = (const double*)llr_dev;
            rc = es ? generic_run_sp64_es(g, x, B, p, bits, soft, iters_used, ws, st, w)
                    : generic_run_sp64(g, x, B, p, bits, soft, iters_used, ws, st, w);
        } else {
            const float* x = (const float*)llr_dev;
            rc = es ? generic_run_sp32_es(g, x, B, p, bits, soft, iters_used, ws, st, w)
                    : generic_run_sp32(g, x, B, p, bits, soft, iters_used, ws, st, w);
        }
    } else if (p.algo == LDPC_ALGO_MIN_SUM) {
        if (p.flags & LDPC_F_F64) return set_error(LDPC_EUNSUPPORTED, "min-sum is float32 only");
        const float* x = (const float*)llr_dev;
        rc = es ? generic_run_ms32_es(g, x, B, p, bits, soft, iters_used, ws, st, w)
                : generic_run_ms32(g, x, B, p, bits, soft, iters_used, ws, st, w);
    } else {
        return set_error(LDPC_EUNSUPPORTED, "algo %d not supported by the generic kernels", p.algo);
    }
    if (rc != LDPC_OK) return rc;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(LDPC_EHIP, "generic kernel launch: %s", hipGetErrorString(e));
    return rc;
}

}  // namespace ldpc
