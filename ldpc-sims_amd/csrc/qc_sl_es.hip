// qc_sl_es.hip — tanh-SP with early termination on the sliced Z = 81 kernel (qc_sl_sp.h), built with the
// default (max-occupancy) scheduler: 2 waves/SIMD without scratch (build.py PER_FILE).
#include "qc_sl_sp.h"

namespace ldpc {

int qc_launch_sp_sl_es_wifi1944_56(const float* llr, int64_t B, const ldpc_params& p, uint8_t* bits, float* soft,
                                   int32_t* used, hipStream_t st) {
    using C = Wifi1944_56;
    const unsigned blocks = (unsigned)((B + 1) / 2);  // the plain pass, then the a == 1 rule's (qc_sl_sp.h PASS)
    hipStream_t s2 = st;
    if (QC_SP_FIXZ) {
        if (const int rc = qc_sp_fork(llr, B, C::NB * C::Z, 2, st, &s2)) return rc;
        k_qc_sp_sl<C, true, 2><<<qc_sp_pass2_grid(blocks), dim3(C::S * 64), 0, s2>>>(llr, B, p.iters, p.clamp, p.flags,
                                                                                      bits, soft, used, qc_sp_zlist());
    }
    k_qc_sp_sl<C, true, QC_SP_FIXZ ? 1 : 0><<<blocks, dim3(C::S * 64), 0, st>>>(llr, B, p.iters, p.clamp, p.flags, bits,
                                                                                soft, used, qc_sp_zlist());
    if (QC_SP_FIXZ)
        if (const int rc = qc_sp_join(st)) return rc;
    return LDPC_OK;
}

}  // namespace ldpc
