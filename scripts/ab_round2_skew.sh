set -o pipefail
export OUT=gpurun_out/ab4
CONFIGS="c1|--steps 33" VARIANTS="build_variants/base.so build_variants/skew40.so build_variants/skew100.so build_variants/base.so build_variants/skew40.so build_variants/skew100.so" bash scripts/ab_configs.sh
