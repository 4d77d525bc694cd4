#!/bin/bash
# A/B kernel builds (build_variants/*.so) with the same bench, one after another in one session.
set -o pipefail
OUT=${OUT:-gpurun_out}; mkdir -p $OUT
ARGS=${ARGS:---steps 33 --warmup 3 --no-cpu-baseline}
for so in ${VARIANTS:-build_variants/*.so}; do
  v=$(basename $so .so)
  LDPC_LIB=$PWD/$so timeout -k 10 300 python bench.py $ARGS > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { echo "variant $v failed"; tail -5 $OUT/ab_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab_$v.json'));print('$v', round(d['value']/1e6,3), 'Mcw/s', round(d['roofline']['launch_ms'],3), 'ms', d['config']['kernel_path'], d['ber']['coded_bler'][4:7])"
done
