set -o pipefail
export OUT=gpurun_out/ab8
CONFIGS="c2|--steps 11 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" VARIANTS="build_variants/head.so build_variants/slB.so build_variants/slA.so build_variants/head.so build_variants/slB.so build_variants/slA.so" bash scripts/ab_configs.sh
