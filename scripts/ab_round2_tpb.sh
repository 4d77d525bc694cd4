#!/bin/bash
# A/B: workgroup size of the register-resident QC kernels (QC_ST_TPB 256 / 128 / 64 threads), headline and
# tanh-SP (648,1/2), alternating builds on one box.
OUT=${OUT:-gpurun_out/ab_tpb} CONFIGS="c1|--steps 22;c1t|--steps 11 --algo tanh" VARIANTS="build_variants/head.so build_variants/tpb128.so build_variants/tpb64.so build_variants/head.so build_variants/tpb128.so build_variants/tpb64.so" bash scripts/ab_configs.sh
