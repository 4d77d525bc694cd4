set -o pipefail
export OUT=gpurun_out/ab12
CONFIGS="c3|--steps 22 --code wifi1296_23 --algo qminsum --iters 20 --ebn0 0:0.5:5;c3es|--steps 22 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5;q648|--steps 22 --algo qminsum --iters 20 --ebn0 0:0.5:5" VARIANTS="build_variants/head.so build_variants/pkil.so build_variants/head.so build_variants/pkil.so" bash scripts/ab_configs.sh
