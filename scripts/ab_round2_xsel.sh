set -o pipefail
export OUT=gpurun_out/ab2
mkdir -p $OUT
LDPC_LIB=$PWD/build_variants/xsel2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "minsum or quantized or qc" > $OUT/pytest_xsel2.log 2>&1 || { echo "tests failed"; tail -20 $OUT/pytest_xsel2.log; exit 1; }
tail -2 $OUT/pytest_xsel2.log
CONFIGS="c1|--steps 33;c3|--steps 22 --code wifi1296_23 --algo qminsum --iters 20 --ebn0 0:0.5:5;c3es|--steps 22 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5" VARIANTS="build_variants/base.so build_variants/xsel2.so build_variants/base.so build_variants/xsel2.so" bash scripts/ab_configs.sh
