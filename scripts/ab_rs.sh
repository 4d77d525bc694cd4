#!/bin/bash
# A/B of the config [2] kernel variants (build_variants/*.so, scripts/mkvariant.sh) on the BASELINE config [2]
# bench leg: each variant first checked bitwise against the generic kernels (scripts/check_variant.py), then
# timed twice, interleaved.  VARIANTS="a b c" bash scripts/ab_rs.sh
set -o pipefail
export TMPDIR=/tmp
V=""
for v in $VARIANTS; do
  LDPC_LIB=$PWD/build_variants/$v.so timeout -k 10 120 python scripts/check_variant.py || { echo "variant $v FAILED the bitwise check"; exit 1; }
  V="$V build_variants/$v.so"
done
OUT=${OUT:-gpurun_out/ab_rs} CONFIGS="c2|--code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768 --no-legs --steps 22" VARIANTS="$V $V" bash scripts/ab_configs.sh
