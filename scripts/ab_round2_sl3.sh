#!/bin/bash
# A/B: sliced tanh-SP (config [2]) with serialized product/sum chains (QC_SL_SP_SERIAL_CN) at 2/3/4 waves,
# L in VGPRs / LDS / global memory, one or two exchange buffers.
OUT=gpurun_out/ab13 CONFIGS="c2|--steps 11 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" VARIANTS="build_variants/head.so build_variants/s2nc.so build_variants/t3nc.so build_variants/t3c.so build_variants/g4c.so build_variants/g3nc.so build_variants/head.so build_variants/t3nc.so build_variants/g4c.so" bash scripts/ab_configs.sh
