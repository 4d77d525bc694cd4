#!/bin/bash
# Profiles of the float register early-stop kernels ((648,1/2) min-sum and tanh-SP, 50 it, early stop).
#   OUT=gpurun_out/<name> bash scripts/gpu_profile_es.sh
set -o pipefail
OUT=${OUT:-gpurun_out/es_prof}; mkdir -p $OUT
OUT=$OUT NAME=es_wifi648_minsum50 KERNEL=k_qc_ms_ph ARGS="--steps 11 --warmup 2 --early-stop" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=es_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--steps 11 --warmup 2 --algo tanh --early-stop" bash scripts/gpu_profile.sh || exit 1
echo done
