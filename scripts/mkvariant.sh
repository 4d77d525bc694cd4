#!/bin/bash
# mkvariant.sh NAME "extra qc.hip flags" : build_variants/NAME.so = the library with qc.hip rebuilt with the flags
set -e
cd "$(dirname "$0")/.."
name=$1; shift
O=ldpc-sims_amd/ldpc_amd/.libldpc_hip.so.objs
mkdir -p build_variants/.o_$name
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function \
  -fno-honor-nans $1 -I include -I ldpc-sims_amd/csrc -c -o build_variants/.o_$name/qc.hip.o ldpc-sims_amd/csrc/qc.hip
hipcc --offload-arch=gfx950 -fPIC -shared -o build_variants/$name.so $O/abi.hip.o $O/generic.hip.o $O/qc_sl.hip.o \
  $O/channel.hip.o build_variants/.o_$name/qc.hip.o
echo build_variants/$name.so
