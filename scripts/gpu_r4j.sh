# fma join (DS_JOIN_FMA): GPU soft trace for scripts/trace_failure.py, then re-profile the two tanh-SP records
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4j; mkdir -p $OUT
timeout -k 10 300 python3 scripts/trace_failure_gpu.py > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
OUT=$OUT NAME=c1_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--algo tanh --clamp 10" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_rs ARGS="--code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
python3 scripts/counters_combine.py $OUT > $OUT/counters.json && echo "combined -> $OUT/counters.json"
