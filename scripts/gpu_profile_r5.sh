#!/bin/bash
# Round 5: profile every BASELINE configuration bench.py reports (the headline, the tanh-SP side number and
# side.configs' three legs) at HEAD on one box and one build; counters are means over one decode per Eb/N0
# point (scripts/gpu_profile.sh), so early-stop records describe the sweep, not one launch.
#   OUT=gpurun_out/<name> bash scripts/gpu_profile_r4.sh
set -o pipefail
OUT=${OUT:-gpurun_out/r5prof}; mkdir -p $OUT
OUT=$OUT NAME=c1_wifi648_minsum50 KERNEL=k_qc_ms_ph ARGS="" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c1_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--algo tanh --clamp 10" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_rs ARGS="--code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c3_wifi1296_q5_20es KERNEL=k_qc_qms_pk ARGS="--code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c4_dvbs2_minsum50 DKERNELS=k_ira_load,k_ira_vn,k_ira_cn,k_ira_out CHUNKS=15 ARGS="--code dvbs2_12 --ebn0 0:0.5:2 --batch 4096" bash scripts/gpu_profile.sh || exit 1
python3 scripts/counters_combine.py $OUT > $OUT/counters.json && echo "combined -> $OUT/counters.json"
