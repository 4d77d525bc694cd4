#!/bin/bash
# A/B: sliced tanh-SP (config [2]) with L of the next column loaded before the current column's chains
# (QC_SL_SP_LPF=1) against the in-order load (0), alternating builds on one box.
OUT=${OUT:-gpurun_out/ab_lpf} CONFIGS="c2|--steps 11 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" VARIANTS="build_variants/slpf0.so build_variants/slpf1.so build_variants/slpf0.so build_variants/slpf1.so" bash scripts/ab_configs.sh
