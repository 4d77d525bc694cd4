# round 5 session p: IRA parity posteriors formed in the check kernel (IRA_CNPAR) — parity and A/B
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5p}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ira.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT CONFIGS="c4|--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-legs" \
  VARIANTS="build_variants/cnpar0.so build_variants/cur.so build_variants/cnpar0.so build_variants/cur.so" bash scripts/ab_configs.sh || exit 1
