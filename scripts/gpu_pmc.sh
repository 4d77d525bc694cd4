#!/bin/bash
# HBM traffic of the decode kernel from PMC counters: FETCH_SIZE and WRITE_SIZE in separate passes
# (they do not fit one TCC pass on gfx950), kernel trace only -- no sys/runtime trace with --pmc.
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:---steps 4 --warmup 1 --no-cpu-baseline}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 bench.py $ARGS > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || { echo "pmc $c failed"; exit 1; }
done
find $OUT -name "*counter_collection.csv" | head
