#!/bin/bash
# Round 6: counter records of every BASELINE configuration bench.py reports, at the shipped library settings (no
# LDPC_* overrides: counters_summary.py rejects a record run with any), via scripts/gpu_profile.sh; PART selects a
# subset so each GPU call stays short: 1 (headline, tanh-SP), 2 (configs [2], [3]), 3 (config [4]), all.
# Config [4] runs as bench times it — two streams, 240 MB Infinity-Cache chunks (35 per 4,096-codeword decode) —
# on 2 Eb/N0 points with 2 timed decodes (a fixed-count decode's work does not depend on the point; the five-point
# PMC passes, ~29 k dispatches, crashed the profiler in round 5); its record's time is the decode's wall span.
#   OUT=gpurun_out/r6prof PART=3 bash scripts/gpu_profile_r6.sh
set -o pipefail
OUT=${OUT:-gpurun_out/r6prof}; mkdir -p $OUT
PART=${PART:-all}
if [ $PART = 1 ] || [ $PART = all ]; then
OUT=$OUT NAME=c1_wifi648_minsum50 KERNEL=k_qc_ms_ph ARGS="" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c1_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--algo tanh --clamp 10" bash scripts/gpu_profile.sh || exit 1
fi
if [ $PART = 2 ] || [ $PART = all ]; then
OUT=$OUT NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_rs ARGS="--code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c3_wifi1296_q5_20es KERNEL=k_qc_qms_pk ARGS="--code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5" bash scripts/gpu_profile.sh || exit 1
fi
if [ $PART = 3 ] || [ $PART = all ]; then
STEPS=2 OUT=$OUT NAME=c4_dvbs2_minsum50 DKERNELS=k_ira_load,k_ira_vn,k_ira_cn,k_ira_out CHUNKS=35 ARGS="--code dvbs2_12 --ebn0 1.5:0.5:2 --batch 4096" bash scripts/gpu_profile.sh || exit 1
fi
if [ $PART = all ]; then
python3 scripts/counters_combine.py $OUT > $OUT/counters.json && echo "combined -> $OUT/counters.json"
fi
