set -o pipefail
export OUT=gpurun_out/ab1
CONFIGS="c2|--steps 11 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" VARIANTS="build_variants/base.so build_variants/sl2.so build_variants/base.so build_variants/sl2.so" bash scripts/ab_configs.sh && \
CONFIGS="c3es|--steps 11 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5;mses|--steps 11 --early-stop" VARIANTS="build_variants/base.so build_variants/es3.so build_variants/base.so build_variants/es3.so" bash scripts/ab_configs.sh && \
CONFIGS="tes|--steps 11 --algo tanh --early-stop" VARIANTS="build_variants/base.so build_variants/es3.so build_variants/es3sp2.so" bash scripts/ab_configs.sh
