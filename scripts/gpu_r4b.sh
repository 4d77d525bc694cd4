#!/bin/bash
# Round 4 session b: config [2] kernel A/B, the config [2] 50-iteration parity test, the GPU soft-output trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
VARIANTS="rsA rsAb10 rsAs2 rsAns rsAs2b10" OUT=gpurun_out/r4b bash scripts/ab_rs.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_config2.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4b/pytest_c2.log 2>&1; tail -6 gpurun_out/r4b/pytest_c2.log
timeout -k 10 300 python scripts/trace_failure_gpu.py
