#!/bin/bash
# Infinity-Cache chunk budget sweep on the generic path (DVB-S2-shaped min-sum/tanh, (1944,5/6) tanh).
set -o pipefail
OUT=${OUT:-gpurun_out}; mkdir -p $OUT
for b in ${BUDGETS:-0 64 128 160 192}; do
  for cfg in "dvbs2s_ms --code dvbs2s_12 --batch 4096 --ebn0 0:0.5:2 --steps 3" \
             "dvbs2s_sp --code dvbs2s_12 --algo tanh --batch 4096 --ebn0 0:0.5:2 --steps 3" \
             "w1944_sp --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768 --steps 5" \
             "w648_ms_gen --force-generic --steps 5"; do
    set -- $cfg; name=$1; shift
    LDPC_CACHE_BUDGET_MB=$b timeout -k 10 200 python bench.py --no-cpu-baseline --warmup 1 "$@" > $OUT/cs_${name}_$b.json 2> $OUT/cs_${name}_$b.err || { echo "$name $b failed"; tail -5 $OUT/cs_${name}_$b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/cs_${name}_$b.json'));print('$name budget=$b', round(d['value']), 'cw/s', round(d['roofline']['launch_ms'],3), 'ms/launch')"
  done
done
