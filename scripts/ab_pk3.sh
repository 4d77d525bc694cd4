# config [3] early-stop packed kernel: workgroup size (QC_PK_TPB_EARLY 128) and fewer address registers
# (QC_PK_ADDR_MIN_USES_Z64 6) re-checked under the phase priorities; parity of each first
set -o pipefail
export TMPDIR=/tmp
B=build_variants
for v in pk_t128 pk_a6; do
  LDPC_LIB=$PWD/$B/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "quantized or packed" > gpurun_out/pk3_$v.log 2>&1 || { echo "parity $v failed"; tail -5 gpurun_out/pk3_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/pk3_$v.log)"
done
OUT=gpurun_out/pk3 CONFIGS="c3|--code wifi1296_23 --algo qminsum --iters 20 --early-stop --qstep 1 --ebn0 0:0.5:5 --no-legs --steps 22 --warmup 11" \
VARIANTS="$B/head.so $B/pk_t128.so $B/pk_a6.so $B/head.so $B/pk_t128.so $B/pk_a6.so" bash scripts/ab_configs.sh
