#!/bin/bash
# Memory-pipeline counters of the IRA kernels (config [4], one stream, so that every dispatch runs alone): TA/TD (the
# CU's address and data units), TCP (vector L1, its TLB), TCC (L2) stall counters, one rocprofv3 pass per group within
# gfx950's per-block limits.  OUT=gpurun_out/ipmc LIBS="base: s8:abvar/s8.so" bash scripts/ira_pmc.sh
set -o pipefail
OUT=${OUT:-gpurun_out/ipmc}; mkdir -p $OUT
export TMPDIR=/tmp LDPC_IRA_STREAMS=1
P1="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"
P2="TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum TD_LOAD_WAVEFRONT_sum TD_SPI_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE"
for v in $LIBS; do
  name=${v%%:*}; lib=${v#*:}
  if [ -n "$lib" ]; then export LDPC_LIB=$lib; else unset LDPC_LIB; fi
  i=0
  for grp in "$P1" "$P2" "$P3"; do
    i=$((i + 1)); d=$OUT/${name}_p$i
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $d -o run -- python3 bench.py --no-cpu-baseline \
      --no-dropin --no-legs --code dvbs2_12 --iters 50 --batch 512 --ebn0 2:0.5:2 --steps 1 --warmup 1 > $d.json 2> $d.err \
      || { echo "$name pass $i failed"; tail -5 $d.err; exit 1; }
    echo "$name pass $i done"
  done
done
