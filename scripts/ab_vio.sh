# packed kernel vectorised I/O (QC_PK_VIO): parity of the in-tree build, then A/B vs QC_PK_VIO=0 on config [3]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "quantized or packed" > gpurun_out/vio_parity.log 2>&1 && tail -2 gpurun_out/vio_parity.log &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bench_legs.py \
    -k config3 > gpurun_out/vio_leg.log 2>&1 && tail -2 gpurun_out/vio_leg.log &&
B=build_variants OUT=gpurun_out/vio \
CONFIGS="es1|--code wifi1296_23 --algo qminsum --iters 1 --early-stop --ebn0 5:0.5:5 --no-legs --steps 20;c3|--code wifi1296_23 --algo qminsum --iters 20 --early-stop --qstep 1 --ebn0 0:0.5:5 --no-legs --steps 3;c3fx|--code wifi1296_23 --algo qminsum --iters 20 --qstep 1 --ebn0 0:0.5:5 --no-legs --steps 3;pk648|--code wifi648_12 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5 --no-legs --steps 3" \
VARIANTS="build_variants/novio.so build_variants/vio.so build_variants/novio.so build_variants/vio.so" bash scripts/ab_configs.sh
