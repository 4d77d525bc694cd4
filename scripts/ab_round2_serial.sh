#!/bin/bash
# A/B: serialized tanh-SP chains — sliced early stop (config [2] with early stop) and the (648,1/2) stored-message
# kernel (fixed and early stop), each against the HEAD library.
set -o pipefail
OUT=gpurun_out/ab14 CONFIGS="c2es|--steps 11 --code wifi1944_56 --algo tanh --early-stop --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" VARIANTS="build_variants/head.so build_variants/se3.so build_variants/se3nc.so build_variants/se2.so build_variants/head.so build_variants/se3.so" bash scripts/ab_configs.sh &&
OUT=gpurun_out/ab14 CONFIGS="t648|--steps 11 --algo tanh;t648es|--steps 11 --algo tanh --early-stop" VARIANTS="build_variants/head.so build_variants/sp4.so build_variants/sp4d.so build_variants/head.so build_variants/sp4.so build_variants/sp4d.so" bash scripts/ab_configs.sh
