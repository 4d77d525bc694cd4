#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_legs.py -x -v --timeout 400 --timeout-method thread > $O/pytest_legs.log 2>&1 || { echo "leg tests failed"; grep -E "FAILED|Error|assert" $O/pytest_legs.log | head; tail -3 $O/pytest_legs.log; exit 1; }
tail -1 $O/pytest_legs.log
OUT=$O VARIANTS="base phX phA4 phA2" bash scripts/ab_ph.sh
