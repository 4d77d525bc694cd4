#!/bin/bash
# Headline-kernel variants (build_variants/*.so): min-sum bit-exact parity first, then 3 interleaved timings.
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/ab_ph}; mkdir -p $O
V=""
for v in $VARIANTS; do
  LDPC_LIB=$PWD/build_variants/$v.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x --timeout 250 -k "minsum_bit_exact" > $O/check_$v.log 2>&1 || { echo "$v FAILED parity"; exit 1; }
  V="$V build_variants/$v.so"
done
OUT=$O CONFIGS="c1|--no-legs --steps 22" VARIANTS="$V $V $V" bash scripts/ab_configs.sh
