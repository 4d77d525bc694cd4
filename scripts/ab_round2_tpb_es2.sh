#!/bin/bash
# GPU tests on the build with one-wave early-stop workgroups, then A/B against the previous head build
# (256-thread workgroups everywhere) on the early-stop configurations, and tanh-SP early stop at 64 (sp64).
set -o pipefail
OUT=${OUT:-gpurun_out/ab_tpb_es2}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
OUT=$OUT CONFIGS="c3es|--steps 11 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5;ms_es|--steps 11 --early-stop;ms1296_es|--steps 11 --code wifi1296_23 --early-stop;sp_es|--steps 11 --algo tanh --early-stop" VARIANTS="build_variants/head.so build_variants/new.so build_variants/sp64.so build_variants/head.so build_variants/new.so build_variants/sp64.so" bash scripts/ab_configs.sh
