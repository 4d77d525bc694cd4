# after idle-lane masking in the headline kernel: re-profile its record, then the full GPU check
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4m; mkdir -p $OUT
OUT=$OUT NAME=c1_wifi648_minsum50 KERNEL=k_qc_ms_ph ARGS="" bash scripts/gpu_profile.sh || exit 1
python3 scripts/counters_combine.py $OUT > $OUT/counters.json && echo "combined -> $OUT/counters.json" &&
bash scripts/gpu_check.sh
