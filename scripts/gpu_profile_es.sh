#!/bin/bash
# Profiles of the float register early-stop kernels ((648,1/2) min-sum and tanh-SP 50 it, (1296,2/3) min-sum 20 it).
#   OUT=gpurun_out/<name> bash scripts/gpu_profile_es.sh
set -o pipefail
OUT=${OUT:-gpurun_out/es_prof}; mkdir -p $OUT
OUT=$OUT NAME=es_wifi648_minsum50 KERNEL=k_qc_ms_ph ARGS="--steps 11 --warmup 2 --early-stop" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=es_wifi1296_minsum20 KERNEL=k_qc_ms_st ARGS="--steps 11 --warmup 2 --early-stop --code wifi1296_23 --iters 20" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=es_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--steps 11 --warmup 2 --algo tanh --early-stop" bash scripts/gpu_profile.sh || exit 1
echo done
