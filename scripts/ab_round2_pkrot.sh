#!/bin/bash
# A/B: packed 5-bit kernel with LDS-row rotations (pkr) vs ds_bpermute (head); GPU tests on the variant first.
set -o pipefail
mkdir -p gpurun_out/ab21
LDPC_LIB=$PWD/build_variants/pkr.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab21/pytest_gpu_pkr.log 2>&1 || { echo "pytest (pkr) failed"; tail -30 gpurun_out/ab21/pytest_gpu_pkr.log; exit 1; }
tail -1 gpurun_out/ab21/pytest_gpu_pkr.log
OUT=gpurun_out/ab21 CONFIGS="c3es|--steps 22 --warmup 0 --code wifi1296_23 --algo qminsum --iters 20 --early-stop;c3|--steps 11 --code wifi1296_23 --algo qminsum --iters 20;q648|--steps 11 --algo qminsum --iters 20;q648es|--steps 11 --algo qminsum --iters 20 --early-stop" VARIANTS="build_variants/head.so build_variants/pkr.so build_variants/head.so build_variants/pkr.so" bash scripts/ab_configs.sh
