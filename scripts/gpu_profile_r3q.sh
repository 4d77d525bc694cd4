#!/bin/bash
# Round-3 third pass: re-profile every register-kernel configuration at HEAD (config [1] min-sum and tanh-SP,
# config [2], config [3] fixed and early stop), one box, one build.
#   OUT=gpurun_out/<name> bash scripts/gpu_profile_r3q.sh
set -o pipefail
OUT=${OUT:-gpurun_out/r3q}; mkdir -p $OUT
OUT=$OUT NAME=c1_wifi648_minsum50 KERNEL=k_qc_ms_ph ARGS="--steps 20 --warmup 3" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c1_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--steps 11 --warmup 2 --algo tanh" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_sl ARGS="--steps 11 --warmup 2 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c3_wifi1296_q5_20es KERNEL=k_qc_qms_pk ARGS="--steps 11 --warmup 2 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c3_wifi1296_q5_20_fixed KERNEL=k_qc_qms_pk ARGS="--steps 11 --warmup 2 --code wifi1296_23 --algo qminsum --iters 20" bash scripts/gpu_profile.sh || exit 1
echo done
