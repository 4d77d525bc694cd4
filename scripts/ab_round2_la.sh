set -o pipefail
export OUT=gpurun_out/ab9
CONFIGS="c1|--steps 33" VARIANTS="build_variants/head.so build_variants/la1.so build_variants/la2.so build_variants/la3.so build_variants/head.so build_variants/la1.so build_variants/la2.so build_variants/la3.so" bash scripts/ab_configs.sh
