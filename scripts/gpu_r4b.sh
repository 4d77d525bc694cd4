#!/bin/bash
# Round 4 session b: config [2] kernel A/B, the full GPU suite (config [2] 50-iteration parity, sweep resume, soft
# parity with the measured failure bounds), the GPU soft-output trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
VARIANTS="rsA rsAb10 rsAs2 rsV rsC8 rsLag rsVLag rsVLagS2 rsDup rsVLagDup" OUT=gpurun_out/r4b bash scripts/ab_rs.sh || exit 1
LDPC_PARITY_LOG=gpurun_out/r4b/soft_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4b/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4b/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4b/pytest_gpu.log
timeout -k 10 300 python scripts/trace_failure_gpu.py
