#!/bin/bash
# A/B: headline phased min-sum with lane rotations through an LDS row (ds_write_addtid_b32 + ds_read_b32) vs
# ds_bpermute; GPU tests against the variant first (bit-exact parity).
set -o pipefail
mkdir -p gpurun_out/ab19
LDPC_LIB=$PWD/build_variants/lr2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab19/pytest_gpu_lr2.log 2>&1 || { echo "pytest (lr) failed"; tail -30 gpurun_out/ab19/pytest_gpu_lr2.log; exit 1; }
tail -1 gpurun_out/ab19/pytest_gpu_lr2.log
OUT=gpurun_out/ab19 CONFIGS="c1|--steps 22" VARIANTS="build_variants/head.so build_variants/lr.so build_variants/lr2.so build_variants/head.so build_variants/lr.so build_variants/lr2.so" bash scripts/ab_configs.sh
