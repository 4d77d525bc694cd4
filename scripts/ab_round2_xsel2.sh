#!/bin/bash
# A/B: compare-free check output in the LDS-row headline kernel (xs) vs HEAD; parity tests on the variant first.
set -o pipefail
mkdir -p gpurun_out/ab23
LDPC_LIB=$PWD/build_variants/xs.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py -x -q --timeout 300 --timeout-method thread -k "minsum or ms or bench_config or qc" > gpurun_out/ab23/pytest_xs.log 2>&1 || { echo "pytest (xs) failed"; tail -30 gpurun_out/ab23/pytest_xs.log; exit 1; }
tail -1 gpurun_out/ab23/pytest_xs.log
OUT=gpurun_out/ab23 CONFIGS="c1|--steps 22" VARIANTS="build_variants/head.so build_variants/xs.so build_variants/head.so build_variants/xs.so build_variants/head.so build_variants/xs.so" bash scripts/ab_configs.sh
