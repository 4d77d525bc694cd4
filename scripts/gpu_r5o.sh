# round 5 session o: price the IRA variable kernel's parity tasks (diagnostic build, wrong results)
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5o}; mkdir -p $OUT
OUT=$OUT CONFIGS="c4|--code dvbs2_12 --iters 50 --batch 4096 --ebn0 1.5:1:1.5 --steps 5 --warmup 1 --no-legs" \
  VARIANTS="build_variants/cur.so build_variants/diag_nopar.so build_variants/cur.so build_variants/diag_nopar.so" bash scripts/ab_configs.sh || exit 1
