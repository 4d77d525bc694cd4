#!/bin/bash
# A/B: workgroup size for the early-stop register kernels — a workgroup's LDS is held until its slowest wave
# exits, so with early stop smaller workgroups free CU slots sooner.  Packed 5-bit kernel (config [3]:
# QC_PK_TPB 256 / 128 / 64) and the (648,1/2) min-sum / tanh-SP early-stop kernels (QC_ST_TPB 256 / 64).
OUT=${OUT:-gpurun_out/ab_tpb_es} CONFIGS="c3es|--steps 11 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5;c3|--steps 11 --code wifi1296_23 --algo qminsum --iters 20" VARIANTS="build_variants/head.so build_variants/pk128.so build_variants/pk64.so build_variants/head.so build_variants/pk128.so build_variants/pk64.so" bash scripts/ab_configs.sh || exit 1
OUT=${OUT:-gpurun_out/ab_tpb_es} CONFIGS="ms_es|--steps 11 --early-stop;sp_es|--steps 11 --algo tanh --early-stop" VARIANTS="build_variants/head.so build_variants/tpb64.so build_variants/head.so build_variants/tpb64.so" bash scripts/ab_configs.sh
