// generic_run.hip — one driver instantiation of the generic decoder (generic_impl.h run<T, MS, ES>), compiled
// once per variant by build.py with RUN_T / RUN_MS / RUN_ES / RUN_NAME defined, so the kernel templates of
// the six variants build in parallel translation units.
#include "generic_impl.h"

namespace ldpc {

int RUN_NAME(const GenericArgs& g, const void* llr, int64_t B, const ldpc_params& p, uint8_t* bits, void* soft,
             int32_t* iters_used, char* ws, hipStream_t st, const BPWeights* w) {
    return run<RUN_T, RUN_MS != 0, RUN_ES != 0>(g, (const RUN_T*)llr, B, p, bits, (RUN_T*)soft, iters_used, ws, st, w);
}

}  // namespace ldpc
