#!/bin/bash
# Round 4: s_setprio phase-priority variants of every register kernel a BASELINE configuration runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_prio2; mkdir -p $O
for v in rsP3 rsP4 rsP1V rsP1C8 rsP1b7; do
  LDPC_LIB=$PWD/build_variants/$v.so timeout -k 10 120 python scripts/check_variant.py || { echo "variant $v FAILED"; exit 1; }
done
for v in phP1 phP2 spP1 spP2 pkP1 pkP2; do
  LDPC_LIB=$PWD/build_variants/$v.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x --timeout 250 -k "minsum_bit_exact or qc_sp_equals or quantized_minsum_vs_oracle or qc_early_stop" > $O/check_$v.log 2>&1 || { echo "variant $v FAILED parity"; tail -5 $O/check_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/check_$v.log)"
done
B=build_variants
OUT=$O CONFIGS="c2|--code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768 --no-legs --steps 22" VARIANTS="$B/base.so $B/rsP3.so $B/rsP4.so $B/rsP1V.so $B/rsP1C8.so $B/rsP1b7.so $B/base.so $B/rsP3.so $B/rsP4.so" bash scripts/ab_configs.sh || exit 1
OUT=$O CONFIGS="c1|--no-legs --steps 22" VARIANTS="$B/base.so $B/phP1.so $B/phP2.so $B/base.so $B/phP1.so $B/phP2.so" bash scripts/ab_configs.sh || exit 1
OUT=$O CONFIGS="t1|--algo tanh --clamp 10 --no-legs --steps 22" VARIANTS="$B/base.so $B/spP1.so $B/spP2.so $B/base.so $B/spP1.so $B/spP2.so" bash scripts/ab_configs.sh || exit 1
OUT=$O CONFIGS="c3|--code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5 --no-legs --steps 22" VARIANTS="$B/base.so $B/pkP1.so $B/pkP2.so $B/base.so $B/pkP1.so $B/pkP2.so" bash scripts/ab_configs.sh || exit 1
