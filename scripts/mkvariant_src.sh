#!/bin/bash
# mkvariant_src.sh NAME FILE SRC "extra flags": abvar/NAME.so = the library with csrc/FILE replaced by SRC (another
# revision of that file, e.g. `git show REV:ldpc-sims_amd/csrc/FILE > /tmp/x.hip`) built with the extra flags; the
# other objects come from the in-tree build.  abvar/ is local only (git- and gpurun-ignored): for an A/B on the GPU
# box build the variant there, `python ldpc-sims_amd/build.py --out build_variants/NAME.so -DKNOB=1`.
set -e
cd "$(dirname "$0")/.."
name=$1; file=$2; src=$3; extra=$4
O=ldpc-sims_amd/ldpc_amd/.libldpc_hip.so.objs
mkdir -p abvar/.o_$name
per=""
case $file in qc.hip|qc_sl.hip) per="-fno-honor-nans -mllvm --amdgpu-sched-strategy=iterative-ilp";; qc_pk.hip|qc_sl_es.hip|qc_es.hip) per="-fno-honor-nans";; esac
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function \
  $per $extra -I include -I ldpc-sims_amd/csrc -c -o abvar/.o_$name/$file.o $src
objs="abvar/.o_$name/$file.o"
for o in $O/*.o; do [ "$(basename $o)" = "$file.o" ] || objs="$objs $o"; done
hipcc --offload-arch=gfx950 -fPIC -shared -o abvar/$name.so $objs
echo abvar/$name.so
