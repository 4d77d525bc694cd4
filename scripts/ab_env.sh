#!/bin/bash
# A/B of environment settings (the library's knobs: LDPC_IRA_*, QC build variants via LDPC_LIB, ...) over one
# bench configuration in one GPU session: each setting runs bench.py once, in the order given.
#   OUT=gpurun_out/ab ARGS="--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1" \
#     SETTINGS="s2b200:LDPC_IRA_STREAMS=2,LDPC_IRA_BUDGET_MB=200;s3b200:LDPC_IRA_STREAMS=3" bash scripts/ab_env.sh
# A setting is NAME:VAR=VALUE[,VAR=VALUE...]; the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/ab}; mkdir -p $OUT
IFS=';' read -ra SETS <<< "$SETTINGS"
for st in "${SETS[@]}"; do
  name=${st%%:*}; vars=${st#*:}
  env_args=(); IFS=',' read -ra KV <<< "$vars"
  for kv in "${KV[@]}"; do env_args+=("$kv"); done
  env "${env_args[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-dropin --no-legs $ARGS > $OUT/ab_$name.json 2> $OUT/ab_$name.err || { echo "$name failed"; tail -5 $OUT/ab_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab_$name.json'));print('$name', round(d['value']), 'cw/s', round(d['roofline']['launch_ms'],3), 'ms', d['config']['kernel_path'])"
done
