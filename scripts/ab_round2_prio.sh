set -o pipefail
export OUT=gpurun_out/ab11
CONFIGS="c1|--steps 33" VARIANTS="build_variants/head.so build_variants/prio1.so build_variants/prio3.so build_variants/amu2.so build_variants/amu4.so build_variants/head.so build_variants/prio1.so build_variants/prio3.so build_variants/amu2.so build_variants/amu4.so" bash scripts/ab_configs.sh
