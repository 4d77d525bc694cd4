#!/bin/bash
# Round 5: counter records of every BASELINE configuration bench.py reports (the headline, the tanh-SP side number,
# side.configs' three legs) at HEAD, via scripts/gpu_profile.sh; PART selects a subset so each GPU call stays short:
#   PART=1 (headline, tanh-SP), PART=2 (configs [2], [3]), PART=3 (config [4]), PART=all.  Then counters_combine.
# Config [4]'s record runs its chunks on ONE stream (LDPC_IRA_STREAMS=1): with two, concurrent dispatches overlap in
# the trace and the per-dispatch counters of the PMC passes (which serialise dispatches) no longer match the timed
# decode; its bytes per decode are the same either way.
#   OUT=gpurun_out/r5prof PART=1 bash scripts/gpu_profile_r5.sh
set -o pipefail
OUT=${OUT:-gpurun_out/r5prof}; mkdir -p $OUT
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
# one Eb/N0 point (a fixed-count decode does the same work at every point): the PMC passes of the five-point grid
# (~29 k dispatches) crashed the profiler (SIGSEGV inside the HIP runtime under --pmc, session r5prof)
# CHUNKS = ceil(4096 / chunk), chunk = (200 MiB / (8n + 16M bytes)) rounded down to 8 = 200 codewords: 21
LDPC_IRA_STREAMS=1 OUT=$OUT NAME=c4_dvbs2_minsum50 DKERNELS=k_ira_load,k_ira_vn,k_ira_cn,k_ira_out CHUNKS=21 ARGS="--code dvbs2_12 --ebn0 1.5:1:1.5 --batch 4096" bash scripts/gpu_profile.sh || exit 1
fi
if [ $PART = all ]; then
python3 scripts/counters_combine.py $OUT > $OUT/counters.json && echo "combined -> $OUT/counters.json"
fi
