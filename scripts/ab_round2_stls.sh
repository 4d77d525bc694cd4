#!/bin/bash
# A/B: LDS-row rotations in the stored min-sum ((1296,2/3) float) and tanh-SP kernels, fixed and early stop.
set -o pipefail
mkdir -p gpurun_out/ab24
LDPC_LIB=$PWD/build_variants/stls.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab24/pytest_stls.log 2>&1 || { echo "pytest (stls) failed"; tail -30 gpurun_out/ab24/pytest_stls.log; exit 1; }
tail -1 gpurun_out/ab24/pytest_stls.log
OUT=gpurun_out/ab24 CONFIGS="f1296|--steps 11 --code wifi1296_23 --algo minsum --iters 20;f1296es|--steps 11 --code wifi1296_23 --algo minsum --iters 20 --early-stop;t648|--steps 11 --algo tanh;t648es|--steps 11 --algo tanh --early-stop;t1296|--steps 5 --code wifi1296_23 --algo tanh" VARIANTS="build_variants/head.so build_variants/stls.so build_variants/head.so build_variants/stls.so" bash scripts/ab_configs.sh
