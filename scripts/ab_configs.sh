#!/bin/bash
# A/B of library variants (build_variants/*.so, scripts/mkvariant.sh) over several bench configurations in
# one GPU session: for each config, every variant back to back.  Chain stops at the first failure.
#   CONFIGS="name1|args1;name2|args2" VARIANTS="build_variants/a.so build_variants/b.so" bash scripts/ab_configs.sh
set -o pipefail
OUT=${OUT:-gpurun_out}; mkdir -p $OUT
IFS=';' read -ra CFGS <<< "$CONFIGS"
for c in "${CFGS[@]}"; do
  name=${c%%|*}; args=${c#*|}
  for so in $VARIANTS; do
    v=$(basename $so .so)
    LDPC_LIB=$PWD/$so timeout -k 10 300 python bench.py --no-cpu-baseline --no-dropin $args > $OUT/ab_${name}_$v.json 2> $OUT/ab_${name}_$v.err || { echo "$name/$v failed"; tail -5 $OUT/ab_${name}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab_${name}_$v.json'));print('$name', '$v', round(d['value']/1e6,3), 'Mcw/s', round(d['roofline']['launch_ms'],3), 'ms', d['config']['kernel_path'])"
  done
done
