#!/bin/bash
# GPU tests, the bench line, an A/B of library variants (round 3: the idle-lane aliasing, Z = 54 packed and
# Z = 81 sliced), the drop-in sweep and a config [2] profile, on one box.  OUT=gpurun_out/<name> bash scripts/gpu_ab_session.sh

set -o pipefail
OUT=${OUT:-gpurun_out/ab_session}; mkdir -p $OUT; export TMPDIR=/tmp
LDPC_PARITY_LOG=$OUT/soft_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', round(d['value']/1e6,3), d['roofline']['bound'], round(d['roofline']['frac'],3), 'dropin', round(d['dropin_cw_per_s']/1e6,3), 'tanh', round(d['side']['gpu_tanh_sp']['cw_per_s']/1e6,3))"
OUT=$OUT CONFIGS="c3es|--steps 22 --warmup 0 --code wifi1296_23 --algo qminsum --iters 20 --early-stop;c3fixed|--steps 11 --warmup 2 --code wifi1296_23 --algo qminsum --iters 20" VARIANTS="build_variants/base.so build_variants/noalias_pk.so build_variants/base.so build_variants/noalias_pk.so" bash scripts/ab_configs.sh || exit 1
OUT=$OUT CONFIGS="c2|--steps 11 --warmup 2 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" VARIANTS="build_variants/base.so build_variants/noalias_sl.so build_variants/base.so build_variants/noalias_sl.so" bash scripts/ab_configs.sh || exit 1
timeout -k 10 300 python scripts/dropin_threads.py > $OUT/dropin_threads.jsonl || { echo dropin sweep failed; exit 1; }
OUT=$OUT NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_sl ARGS="--steps 11 --warmup 2 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh || exit 1
echo done
