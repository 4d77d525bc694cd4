#!/bin/bash
# Profiling sessions (one gpurun call: the bench number, kernel stats and counters come from one box) (scripts/gpu_profile.sh) for the headline and the register-kernel configurations;
# combine with: python scripts/counters_combine.py gpurun_out/<dir> > profiles/counters.json
set -o pipefail
export OUT=${OUT:-gpurun_out}
NAME=c1_wifi648_minsum50 KERNEL=k_qc_ms_ph ARGS="--steps 22 --warmup 3" bash scripts/gpu_profile.sh || exit 1
NAME=c1_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--steps 11 --warmup 2 --algo tanh" bash scripts/gpu_profile.sh || exit 1
NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_sl ARGS="--steps 11 --warmup 2 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
NAME=c3_wifi1296_q5_20es KERNEL=k_qc_qms_pk ARGS="--steps 22 --warmup 0 --code wifi1296_23 --algo qminsum --iters 20 --early-stop" PARGS="--steps 11 --warmup 0" bash scripts/gpu_profile.sh || exit 1
NAME=c3_wifi1296_q5_20_fixed KERNEL=k_qc_qms_pk ARGS="--steps 11 --warmup 2 --code wifi1296_23 --algo qminsum --iters 20" bash scripts/gpu_profile.sh || exit 1
