#!/bin/bash
# A/B: LDS-row rotations (lr2) with rotation lookahead 2 / 3 and address registers for shifts used >= 4 times.
set -o pipefail
OUT=gpurun_out/ab20 CONFIGS="c1|--steps 22" VARIANTS="build_variants/head.so build_variants/lr2.so build_variants/la2.so build_variants/la3.so build_variants/am4.so build_variants/head.so build_variants/lr2.so build_variants/la2.so build_variants/la3.so build_variants/am4.so" bash scripts/ab_configs.sh
