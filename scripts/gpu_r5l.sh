# round 5 session l: IRA check states as 12-byte records (one dwordx3 per state) — parity and A/B vs split arrays
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5l}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ira.py tests/test_gpu_multirank.py -k "ira or dvbs2 or config4 or Ira or IRA" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT CONFIGS="c4|--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-legs" \
  VARIANTS="build_variants/split.so build_variants/cur.so build_variants/split.so build_variants/cur.so" bash scripts/ab_configs.sh || exit 1
OUT=$OUT/kp NAME=c4 ARGS="--code dvbs2_12 --batch 4096 --ebn0 1.5:1:1.5 --steps 2 --warmup 1" LDPC_IRA_STREAMS=1 bash scripts/kprof.sh > /dev/null || exit 1
head -2 $OUT/kp/c4/summary.txt | cut -c1-200
