#!/bin/bash
# A/B: occupancy of the spilling non-BASELINE register kernels — (1296,2/3) float min-sum k_qc_ms_st at 3
# waves/SIMD (spill-free) and (648,1/2) 5-bit packed k_qc_qms_pk at 3 / 2 (early stop) waves (spill-free).
set -o pipefail
OUT=gpurun_out/ab16 CONFIGS="f1296|--steps 11 --code wifi1296_23 --algo minsum --iters 20;f1296es|--steps 11 --code wifi1296_23 --algo minsum --iters 20 --early-stop" VARIANTS="build_variants/head.so build_variants/st3.so build_variants/head.so build_variants/st3.so" bash scripts/ab_configs.sh &&
OUT=gpurun_out/ab16 CONFIGS="q648|--steps 11 --algo qminsum --iters 20;q648es|--steps 11 --algo qminsum --iters 20 --early-stop" VARIANTS="build_variants/head.so build_variants/pk32.so build_variants/head.so build_variants/pk32.so" bash scripts/ab_configs.sh
