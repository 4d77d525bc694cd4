#!/bin/bash
# GPU tests + A/B of tanh-SP library variants (build_variants/*.so) against the in-tree build.
#   OUT=gpurun_out/<name> VARIANTS="build_variants/a.so ..." bash scripts/gpu_r3j.sh
set -o pipefail
OUT=${OUT:-gpurun_out/r3j}; mkdir -p $OUT; export TMPDIR=/tmp
LDPC_PARITY_LOG=$OUT/soft_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 1 -o $rc -eq 0 ] || exit 1
OUT=$OUT CONFIGS="tanh648|--steps 11 --warmup 2 --algo tanh;c2|--steps 11 --warmup 2 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768;tanh648es|--steps 11 --warmup 2 --algo tanh --early-stop" VARIANTS="$VARIANTS" bash scripts/ab_configs.sh
