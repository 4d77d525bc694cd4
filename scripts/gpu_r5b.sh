# round 5 session b: parity of the interleaved packed kernel and the config [2] changes, A/B of both, IRA profile
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5b}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_config2.py tests/test_gpu_bench_legs.py -k "packed or qms or quantized or zero or config2 or config3 or resident or kernels_agree" > $OUT/pytest.log 2>&1; rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT CONFIGS="c2|--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 4:0.5:9 --no-legs --steps 11 --warmup 3" \
  VARIANTS="build_variants/c2_r4like.so build_variants/c2_fix0.so build_variants/c2_pos0.so build_variants/cur.so build_variants/c2_r4like.so build_variants/c2_fix0.so build_variants/c2_pos0.so build_variants/cur.so" bash scripts/ab_configs.sh || exit 1
OUT=$OUT CONFIGS="c3|--code wifi1296_23 --algo qminsum --iters 20 --batch 65536 --early-stop --ebn0 0:0.5:5 --no-legs --steps 22 --warmup 3" \
  VARIANTS="build_variants/c3_ilv0.so build_variants/cur.so build_variants/c3_ilv0.so build_variants/cur.so" bash scripts/ab_configs.sh || exit 1
OUT=$OUT/kp NAME=c4ira ARGS="--code dvbs2_12 --batch 4096 --ebn0 1.5:1:1.5 --steps 2 --warmup 1" bash scripts/kprof.sh
