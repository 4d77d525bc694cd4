#!/bin/bash
# mkvariant.sh NAME FILE "extra flags" : build_variants/NAME.so = the library with csrc/FILE rebuilt with the
# extra flags (other objects from the in-tree build; run `python ldpc-sims_amd/build.py` first)
set -e
cd "$(dirname "$0")/.."
name=$1; file=$2; extra=$3
O=ldpc-sims_amd/ldpc_amd/.libldpc_hip.so.objs
mkdir -p build_variants/.o_$name
per=""
case $file in qc.hip|qc_sl.hip) per="-fno-honor-nans -mllvm --amdgpu-sched-strategy=iterative-ilp";; qc_pk.hip|qc_sl_es.hip) per="-fno-honor-nans";; esac
[ -n "$NOSCHED" ] && per="-fno-honor-nans"   # default (max-occupancy) scheduler
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function \
  $per $extra -I include -I ldpc-sims_amd/csrc -c -o build_variants/.o_$name/$file.o ldpc-sims_amd/csrc/$file
objs="build_variants/.o_$name/$file.o"
for o in $O/*.o; do [ "$(basename $o)" = "$file.o" ] || objs="$objs $o"; done
hipcc --offload-arch=gfx950 -fPIC -shared -o build_variants/$name.so $objs
echo build_variants/$name.so
