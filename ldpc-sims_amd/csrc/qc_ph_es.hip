// qc_ph_es.hip — the float early-stop phased min-sum kernels (k_qc_ms_ph<C, false, true, N>, Z <= 32) in a
// translation unit of their own, built with the default scheduler (build.py): qc.hip's other kernels use
// iterative-ILP scheduling, under which this kernel's row-wise syndrome spills.  The kernel template is
// qc.hip's; QC_TU_PH_ES keeps everything but this launcher out of this unit.
#define QC_TU_PH_ES 1
#include "qc.hip"
