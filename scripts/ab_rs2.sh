# config [2] check-row block size after the fma join (QC_RS_DS_BLOCK; blocks give bitwise-equal outputs):
# parity of the shipped build, then A/B: join1 = blocks of 10 (before), head = 20 (one block), rs_b14, rs_b16
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python scripts/check_variant.py > gpurun_out/rs2_check.log 2>&1 && tail -1 gpurun_out/rs2_check.log &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_config2.py tests/test_gpu_bench_legs.py -k "config2" > gpurun_out/rs2_tests.log 2>&1 && tail -1 gpurun_out/rs2_tests.log &&
OUT=gpurun_out/rs2 CONFIGS="c2|--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 4:0.5:9 --no-legs --steps 11 --warmup 3" \
VARIANTS="build_variants/join1.so build_variants/head.so build_variants/rs_b14.so build_variants/rs_b16.so build_variants/join1.so build_variants/head.so build_variants/rs_b14.so build_variants/rs_b16.so" bash scripts/ab_configs.sh
