# headline kernel (k_qc_ms_ph) variants re-checked with the phase priorities: APP broadcast (QC_PH_APPB, with
# and without lookahead) and the compare-free select (QC_PH_XSEL)
set -o pipefail
export TMPDIR=/tmp
B=build_variants
OUT=gpurun_out/ph2 CONFIGS="c1|--no-legs --steps 22 --warmup 3" \
VARIANTS="$B/head.so $B/ph_appb.so $B/ph_appb0.so $B/ph_xsel.so $B/head.so $B/ph_appb.so $B/ph_appb0.so $B/ph_xsel.so" bash scripts/ab_configs.sh
