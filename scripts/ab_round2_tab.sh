set -o pipefail
export OUT=gpurun_out/ab10
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
CONFIGS="c1|--steps 33;c1t|--steps 11 --algo tanh;c3es|--steps 22 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5;c3|--steps 22 --code wifi1296_23 --algo qminsum --iters 20 --ebn0 0:0.5:5;c2|--steps 11 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" VARIANTS="build_variants/la1old.so build_variants/newtab.so build_variants/la1old.so build_variants/newtab.so" bash scripts/ab_configs.sh
