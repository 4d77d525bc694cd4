set -o pipefail
export OUT=gpurun_out/ab6
CONFIGS="c1|--steps 33" VARIANTS="build_variants/head.so build_variants/comp.so build_variants/st.so build_variants/head.so build_variants/comp.so build_variants/st.so" bash scripts/ab_configs.sh
