# config [2] with one-block check rows: re-profile its counter record
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4k; mkdir -p $OUT
OUT=$OUT NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_rs ARGS="--code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
python3 scripts/counters_combine.py $OUT > $OUT/counters.json && echo "combined -> $OUT/counters.json"
