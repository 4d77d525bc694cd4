#!/bin/bash
# Round refresh in one GPU session: parity tests + smoke + bench + rocprof stats (gpu_round.sh), one bench
# line per BASELINE config (bench_configs.sh), PMC HBM traffic of the headline kernel (gpu_pmc.sh) and
# SQ counters of the stored min-sum kernel (gpu_sq.sh).  Stops at the first failing step.
set -o pipefail
export OUT=${OUT:-gpurun_out}
bash scripts/gpu_round.sh || exit 1
bash scripts/bench_configs.sh || exit 1
bash scripts/gpu_pmc.sh || exit 1
python3 scripts/pmc_summary.py $OUT --kernel k_qc_ms_st --dest $OUT/pmc_traffic.json || exit 1
KERNEL=k_qc_ms_st COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY|SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA|SQ_IFETCH SQC_ICACHE_BUSY_CYCLES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
  bash scripts/gpu_sq.sh > $OUT/sq_counters.txt || exit 1
cat $OUT/sq_counters.txt
