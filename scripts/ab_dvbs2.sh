#!/bin/bash
# A/B of generic-kernel library variants on BASELINE config [4] (DVB-S2 64800 rate 1/2, min-sum 50 it, B = 4096):
# each variant first passes the DVB-S2 parity tests (bitwise vs the oracle), then is timed twice, interleaved.
#   VARIANTS="base skip" bash scripts/ab_dvbs2.sh
set -o pipefail
export TMPDIR=/tmp
V=""
for v in $VARIANTS; do
  LDPC_LIB=$PWD/build_variants/$v.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -k "dvbs2 or minsum_bit_exact" --timeout 250 > gpurun_out/ab_dvbs2_check_$v.log 2>&1 || { echo "variant $v FAILED parity"; tail -5 gpurun_out/ab_dvbs2_check_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/ab_dvbs2_check_$v.log)"
  V="$V build_variants/$v.so"
done
OUT=${OUT:-gpurun_out/ab_dvbs2} CONFIGS="c4|--code dvbs2_12 --batch 4096 --ebn0 0:0.5:2 --no-legs --steps 10 --warmup 1" VARIANTS="$V $V" bash scripts/ab_configs.sh
