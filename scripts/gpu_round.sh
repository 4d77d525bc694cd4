#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.  Every GPU step has its own
# time limit and the chain stops at the first failure (no retries).
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
export TMPDIR=/tmp
STEPS=${STEPS:-22}
rm -f $OUT/soft_parity.jsonl
LDPC_PARITY_LOG=$OUT/soft_parity.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo rocprof failed; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
