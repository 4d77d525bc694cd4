// qc_es.hip — the early-stop register kernels for Z <= 64 (float min-sum: k_qc_ms_ph<C, false, true, N> for
// Z <= 32, k_qc_ms_st<C, false, true, N> above; tanh-SP: k_qc_sp_st<C, true>) in a translation unit of their
// own, built with the default scheduler (build.py): qc.hip's fixed-count kernels use iterative-ILP scheduling,
// under which these kernels' row-wise syndromes spill.  The kernel templates are qc.hip's; QC_TU_ES keeps
// everything but the early-stop launchers out of this unit.
#define QC_TU_ES 1
#include "qc.hip"
