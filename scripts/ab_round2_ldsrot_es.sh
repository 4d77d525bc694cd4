#!/bin/bash
# A/B: phased min-sum early stop with LDS-row rotations (M0 set once) vs ds_bpermute.
set -o pipefail
OUT=gpurun_out/ab22 CONFIGS="c1es|--steps 22 --early-stop" VARIANTS="build_variants/head.so build_variants/lre.so build_variants/head.so build_variants/lre.so" bash scripts/ab_configs.sh
