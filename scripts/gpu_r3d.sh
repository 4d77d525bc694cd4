#!/bin/bash
# Round-3 check: GPU tests, drop-in thread sweep, config [3] and tanh-SP lines and profiles on one box.
set -o pipefail
OUT=${OUT:-gpurun_out/r3d}; mkdir -p $OUT; export TMPDIR=/tmp
LDPC_PARITY_LOG=$OUT/soft_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python scripts/dropin_threads.py > $OUT/dropin_threads.jsonl || { echo dropin sweep failed; exit 1; }
OUT=$OUT NAME=c3_wifi1296_q5_20es KERNEL=k_qc_qms_pk ARGS="--steps 22 --warmup 0 --code wifi1296_23 --algo qminsum --iters 20 --early-stop" PARGS="--steps 11 --warmup 0" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c3_wifi1296_q5_20_fixed KERNEL=k_qc_qms_pk ARGS="--steps 11 --warmup 2 --code wifi1296_23 --algo qminsum --iters 20" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c1_wifi648_tanh50 KERNEL=k_qc_sp_st ARGS="--steps 11 --warmup 2 --algo tanh" bash scripts/gpu_profile.sh || exit 1
OUT=$OUT NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_sl ARGS="--steps 11 --warmup 2 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
echo done
