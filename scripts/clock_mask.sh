# same-box clock of the headline kernel with and without idle-lane masking (GRBM_GUI_ACTIVE over the traced
# duration, scripts/counters_summary.py): evidence for the power-limit reading of DESIGN §3.2
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/clock; mkdir -p $OUT
LDPC_LIB=$PWD/build_variants/ph_nomask.so OUT=$OUT NAME=c1_nomask KERNEL=k_qc_ms_ph ARGS="" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c1_mask KERNEL=k_qc_ms_ph ARGS="" bash scripts/gpu_profile.sh || exit 1
LDPC_LIB=$PWD/build_variants/ph_nomask.so OUT=$OUT NAME=c1_nomask2 KERNEL=k_qc_ms_ph ARGS="" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c1_mask2 KERNEL=k_qc_ms_ph ARGS="" bash scripts/gpu_profile.sh || exit 1
