# idle lanes EXEC-masked out of the tanh-SP iteration loops (QC_SP_MASK_IDLE: (648,1/2) register kernel;
# QC_RS_MASK_IDLE: config [2] resident kernel; QC_PK_MASK_IDLE: packed 5-bit kernels, config [3]) vs head (= shipped, headline masking on); parity first
set -o pipefail
export TMPDIR=/tmp
B=build_variants
LDPC_LIB=$PWD/$B/rs_mask.so timeout -k 10 300 python scripts/check_variant.py > gpurun_out/mask2_check.log 2>&1 && tail -1 gpurun_out/mask2_check.log &&
LDPC_LIB=$PWD/$B/rs_mask.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_config2.py > gpurun_out/mask2_c2.log 2>&1 && tail -1 gpurun_out/mask2_c2.log &&
LDPC_LIB=$PWD/$B/pk_mask.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "quantized or packed" > gpurun_out/mask2_pk.log 2>&1 && tail -1 gpurun_out/mask2_pk.log &&
LDPC_LIB=$PWD/$B/pk_mask.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bench_legs.py -k config3 > gpurun_out/mask2_pkleg.log 2>&1 && tail -1 gpurun_out/mask2_pkleg.log &&
LDPC_LIB=$PWD/$B/sp_mask.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_soft_parity.py -k "wifi648 and auto" > gpurun_out/mask2_sp.log 2>&1 && tail -1 gpurun_out/mask2_sp.log &&
OUT=gpurun_out/mask2 CONFIGS="c1tanh|--code wifi648_12 --algo tanh --iters 50 --clamp 10 --no-legs --steps 11 --warmup 3;c2|--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 4:0.5:9 --no-legs --steps 11 --warmup 3;c3|--code wifi1296_23 --algo qminsum --iters 20 --early-stop --qstep 1 --ebn0 0:0.5:5 --no-legs --steps 22 --warmup 11" \
VARIANTS="$B/head.so $B/sp_mask.so $B/rs_mask.so $B/pk_mask.so $B/head.so $B/sp_mask.so $B/rs_mask.so $B/pk_mask.so" bash scripts/ab_configs.sh
