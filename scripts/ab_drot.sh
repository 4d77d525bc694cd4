# packed 5-bit kernel: doubled-row LDS rotations (QC_PK_DROT / _EARLY) vs ds_bpermute; parity of the variant
# (every packed / quantized test through LDPC_LIB), then A/B on config [3] and the fixed count / (648,1/2)
set -o pipefail
export TMPDIR=/tmp
B=build_variants
LDPC_LIB=$PWD/$B/pk_dr.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "quantized or packed" > gpurun_out/drot_parity.log 2>&1 && tail -1 gpurun_out/drot_parity.log &&
LDPC_LIB=$PWD/$B/pk_dr.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bench_legs.py \
    -k config3 > gpurun_out/drot_leg.log 2>&1 && tail -1 gpurun_out/drot_leg.log &&
OUT=gpurun_out/drot CONFIGS="c3|--code wifi1296_23 --algo qminsum --iters 20 --early-stop --qstep 1 --ebn0 0:0.5:5 --no-legs --steps 22 --warmup 11;c3fx|--code wifi1296_23 --algo qminsum --iters 20 --qstep 1 --ebn0 0:0.5:5 --no-legs --steps 11 --warmup 3;pk648es|--code wifi648_12 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5 --no-legs --steps 22 --warmup 11" \
VARIANTS="$B/head.so $B/pk_dre.so $B/pk_dr.so $B/head.so $B/pk_dre.so $B/pk_dr.so" bash scripts/ab_configs.sh
