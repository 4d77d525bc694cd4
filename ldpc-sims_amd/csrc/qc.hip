// qc.hip — structure-specialised quasi-cyclic decoders (placeholder: none compiled yet).
#include "common.h"
namespace ldpc {
struct QCSpec { int mb, nb, z; };
const QCSpec* qc_lookup(int, int, int, const int32_t*) { return nullptr; }
int qc_z(const QCSpec* s) { return s ? s->z : 0; }
bool qc_supports(const QCSpec*, const ldpc_params&) { return false; }
size_t qc_workspace(const QCSpec*, int64_t, const ldpc_params&) { return 0; }
int qc_decode(const QCSpec*, const void*, int64_t, const ldpc_params&, uint8_t*, void*, int32_t*, char*, hipStream_t) {
    return set_error(LDPC_EUNSUPPORTED, "no QC kernel");
}
}  // namespace ldpc
