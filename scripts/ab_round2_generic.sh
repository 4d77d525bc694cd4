#!/bin/bash
# A/B: generic tanh-SP kernels with slot loops by static_for (no scratch for the V = 2, MAXD 12/16 variants)
# against the previous build, then the GPU tests on the new build.
set -o pipefail
OUT=gpurun_out/ab15 CONFIGS="g1296t|--steps 5 --code wifi1296_23 --algo tanh --force-generic;g1296tes|--steps 5 --code wifi1296_23 --algo tanh --force-generic --early-stop" VARIANTS="build_variants/genold.so build_variants/gennew.so build_variants/genold.so build_variants/gennew.so" bash scripts/ab_configs.sh &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab15/pytest_gpu.log 2>&1 && tail -1 gpurun_out/ab15/pytest_gpu.log
