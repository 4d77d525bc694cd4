#!/bin/bash
# mkvariant_gen.sh NAME "extra flags": build_variants/NAME.so = the library with the fp32 min-sum generic driver
# (generic_run_ms32.o: generic_run.hip, RUN_T=float RUN_MS=1 RUN_ES=0) rebuilt with the extra flags
set -e
cd "$(dirname "$0")/.."
name=$1; extra=$2
O=ldpc-sims_amd/ldpc_amd/.libldpc_hip.so.objs
mkdir -p build_variants/.o_$name
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function \
  -DRUN_T=float -DRUN_MS=1 -DRUN_ES=0 -DRUN_NAME=generic_run_ms32 $extra -I include -I ldpc-sims_amd/csrc \
  -c -o build_variants/.o_$name/generic_run_ms32.o ldpc-sims_amd/csrc/generic_run.hip
objs="build_variants/.o_$name/generic_run_ms32.o"
for o in $O/*.o; do [ "$(basename $o)" = "generic_run_ms32.o" ] || objs="$objs $o"; done
hipcc --offload-arch=gfx950 -fPIC -shared -o build_variants/$name.so $objs
echo build_variants/$name.so
