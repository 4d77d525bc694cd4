# headline: idle lanes EXEC-masked out of the iteration loop (QC_PH_MASK_IDLE) — the LDS/VALU-heavy kernel runs at a
# lower clock than the others on the same box (profiles/counters.json: 2.23 vs 2.38-2.40 GHz), i.e. power-limited;
# parity (bitwise vs the oracle on the bench config) first
set -o pipefail
export TMPDIR=/tmp
B=build_variants
LDPC_LIB=$PWD/$B/ph_mask.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bench_config.py tests/test_gpu_parity.py -k "bench or minsum or ragged" > gpurun_out/mask_parity.log 2>&1 && tail -1 gpurun_out/mask_parity.log &&
OUT=gpurun_out/mask CONFIGS="c1|--no-legs --steps 22 --warmup 3" \
VARIANTS="$B/head.so $B/ph_mask.so $B/head.so $B/ph_mask.so $B/head.so $B/ph_mask.so" bash scripts/ab_configs.sh
