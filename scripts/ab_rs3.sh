# config [2] after one-block check rows: two outputs in flight per row (QC_RS_ROW_LAG 1, one block / blocks of 14)
# and the row-gather priority (QC_RS_PRIO 3); check_variant on the lag builds first
set -o pipefail
export TMPDIR=/tmp
B=build_variants
for v in rs_lag rs_lag14; do
  LDPC_LIB=$PWD/$B/$v.so timeout -k 10 300 python scripts/check_variant.py > gpurun_out/rs3_$v.log 2>&1 || { echo "check $v failed"; tail -3 gpurun_out/rs3_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/rs3_$v.log)"
done
OUT=gpurun_out/rs3 CONFIGS="c2|--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 4:0.5:9 --no-legs --steps 11 --warmup 3" \
VARIANTS="$B/head.so $B/rs_lag.so $B/rs_lag14.so $B/rs_p3.so $B/head.so $B/rs_lag.so $B/rs_lag14.so $B/rs_p3.so" bash scripts/ab_configs.sh
