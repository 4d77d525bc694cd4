set -o pipefail
export OUT=gpurun_out/ab3
CONFIGS="c1|--steps 33" VARIANTS="build_variants/base.so build_variants/sch6.so build_variants/sch4.so build_variants/base.so build_variants/sch6.so build_variants/sch4.so" bash scripts/ab_configs.sh
