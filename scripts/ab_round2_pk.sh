set -o pipefail
export OUT=gpurun_out/ab5
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
CONFIGS="c3|--steps 22 --code wifi1296_23 --algo qminsum --iters 20 --ebn0 0:0.5:5;c3es|--steps 22 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5;q648|--steps 22 --algo qminsum --iters 20 --ebn0 0:0.5:5;q648es|--steps 22 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5" VARIANTS="build_variants/base.so build_variants/pk.so build_variants/base.so build_variants/pk.so" bash scripts/ab_configs.sh
