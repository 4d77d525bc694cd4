# config [2]: qc_sl.hip built with other LLVM AMDGPU scheduling strategies (default / max-ilp) vs the shipped
# iterative-ILP build; check_variant on each first
set -o pipefail
export TMPDIR=/tmp
B=build_variants
for v in sc_def sc_max-ilp; do
  LDPC_LIB=$PWD/$B/$v.so timeout -k 10 300 python scripts/check_variant.py > gpurun_out/sched_$v.log 2>&1 || { echo "check $v failed"; tail -3 gpurun_out/sched_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/sched_$v.log)"
done
OUT=gpurun_out/sched CONFIGS="c2|--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 4:0.5:9 --no-legs --steps 11 --warmup 3" \
VARIANTS="$B/head.so $B/sc_def.so $B/sc_max-ilp.so $B/head.so $B/sc_def.so $B/sc_max-ilp.so" bash scripts/ab_configs.sh
