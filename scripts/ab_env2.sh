#!/bin/bash
# Interleaved A/B of environment settings: ROUNDS passes over SETTINGS (as scripts/ab_env.sh), so box drift
# shows as spread within a setting instead of a difference between settings.  One line per run, summary at the end.
#   OUT=gpurun_out/ab ROUNDS=2 ARGS="..." SETTINGS="a:LDPC_X=1;b:LDPC_X=2" bash scripts/ab_env2.sh
set -o pipefail
OUT=${OUT:-gpurun_out/ab}; mkdir -p $OUT
ROUNDS=${ROUNDS:-2}
IFS=';' read -ra SETS <<< "$SETTINGS"
for r in $(seq 1 $ROUNDS); do
for st in "${SETS[@]}"; do
  name=${st%%:*}; vars=${st#*:}
  env_args=(); IFS=',' read -ra KV <<< "$vars"
  for kv in "${KV[@]}"; do env_args+=("$kv"); done
  env "${env_args[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-dropin --no-legs $ARGS > $OUT/ab_${name}_$r.json 2> $OUT/ab_${name}_$r.err || { echo "$name failed"; tail -5 $OUT/ab_${name}_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab_${name}_$r.json'));c=d.get('clock') or {};print('$name', $r, round(d['value']), 'cw/s', round(d['roofline']['launch_ms'],3), 'ms', d['config']['kernel_path'], 'clk', round(c.get('clock_mhz',0)), c.get('error',''))" | tee -a $OUT/summary.txt
done
done
