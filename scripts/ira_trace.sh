#!/bin/bash
# Kernel traces of config [4] (DVB-S2 1/2 min-sum 50 it, B = 4,096, one Eb/N0 point) for library variants and stream
# counts: OUT=gpurun_out/kt VARIANTS="base: s8:abvar/s8.so" STREAMS="1 2" bash scripts/ira_trace.sh
# (a variant is NAME:LIBRARY, empty library = the in-tree build); summarise with scripts/ira_trace_summary.py.
set -o pipefail
OUT=${OUT:-gpurun_out/kt}; mkdir -p $OUT
for v in $VARIANTS; do
  name=${v%%:*}; lib=${v#*:}
  for st in $STREAMS; do
    d=$OUT/${name}_st$st
    if [ -n "$lib" ]; then export LDPC_LIB=$lib; else unset LDPC_LIB; fi
    export LDPC_IRA_STREAMS=$st
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --no-cpu-baseline \
      --no-dropin --no-legs --code dvbs2_12 --iters 50 --batch ${BATCH:-4096} --ebn0 2:0.5:2 --steps 2 --warmup 1 > $d.json 2> $d.err \
      || { echo "$name st$st failed"; tail -5 $d.err; exit 1; }
    f=$(find $d -name "*kernel_trace.csv" | head -1); gzip -f "$f"
    echo "$name st$st done"
  done
done
