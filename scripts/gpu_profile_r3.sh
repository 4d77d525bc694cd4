#!/bin/bash
# Round-3 second-pass profiles: the headline and the two tanh-SP configurations whose kernels changed.
#   OUT=gpurun_out/<name> bash scripts/gpu_profile_r3.sh
set -o pipefail
OUT=${OUT:-gpurun_out/r3prof2}; mkdir -p $OUT
OUT=$OUT NAME=c1_wifi648_minsum50 KERNEL=k_qc_ms_ph ARGS="--steps 20 --warmup 3" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c1_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--steps 11 --warmup 2 --algo tanh" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_sl ARGS="--steps 11 --warmup 2 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
echo done
