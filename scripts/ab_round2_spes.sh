#!/bin/bash
# A/B: serial chains in the (1296,2/3) tanh-SP early-stop kernel (spill-free) vs HEAD; then the GPU tests.
set -o pipefail
OUT=gpurun_out/ab17 CONFIGS="t1296es|--steps 11 --code wifi1296_23 --algo tanh --early-stop --ebn0 1:0.5:6" VARIANTS="build_variants/head.so build_variants/spes.so build_variants/head.so build_variants/spes.so" bash scripts/ab_configs.sh &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab17/pytest_gpu.log 2>&1 && tail -1 gpurun_out/ab17/pytest_gpu.log
