# round 5 session h: config [4] A/B of the IRA kernels before / after the batched-load restructure (same box)
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5h}; mkdir -p $OUT
OUT=$OUT CONFIGS="c4|--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-legs" \
  VARIANTS="build_variants/ira_old.so build_variants/cur.so build_variants/ira_old.so build_variants/cur.so" bash scripts/ab_configs.sh || exit 1
OUT=$OUT/kp NAME=c4 ARGS="--code dvbs2_12 --batch 4096 --ebn0 1.5:1:1.5 --steps 2 --warmup 1" bash scripts/kprof.sh > /dev/null || exit 1
head -2 $OUT/kp/c4/summary.txt | cut -c1-200
