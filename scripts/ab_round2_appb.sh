#!/bin/bash
# APP broadcast in the phased min-sum kernel (QC_PH_APPB): GPU tests on the variant, then A/B against the
# head build on the headline configuration, alternating on one box.
set -o pipefail
OUT=${OUT:-gpurun_out/ab_appb}; mkdir -p $OUT
LDPC_LIB=$PWD/build_variants/appb0la.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_appb0la.log 2>&1 || { echo "pytest on appb0la failed"; tail -30 $OUT/pytest_appb0la.log; exit 1; }
tail -1 $OUT/pytest_appb0la.log
OUT=$OUT CONFIGS="c1|--steps 22" VARIANTS="build_variants/head.so build_variants/appb0la.so build_variants/appb1.so build_variants/head.so build_variants/appb0la.so build_variants/head.so build_variants/appb0la.so" bash scripts/ab_configs.sh
