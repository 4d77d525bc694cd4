# config [4] generic streaming kernels: tile shape knobs (GEN_TPL2_MAX threads per node, GEN_VW_CAP codewords per
# thread) vs the shipped 256 threads x 4 codewords; parity of each variant on the DVB-S2 min-sum test first
set -o pipefail
export TMPDIR=/tmp
B=build_variants
for v in g_t6 g_t7 g_v2 g_v2t7; do
  LDPC_LIB=$PWD/$B/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
      -k "dvbs2" > gpurun_out/gen_$v.log 2>&1 || { echo "parity $v failed"; tail -5 gpurun_out/gen_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/gen_$v.log)"
done
OUT=gpurun_out/gen CONFIGS="c4|--code dvbs2_12 --algo minsum --iters 50 --batch 4096 --ebn0 0:0.5:2 --no-legs --no-dropin --steps 5 --warmup 2" \
VARIANTS="$B/head.so $B/g_t6.so $B/g_t7.so $B/g_v2.so $B/g_v2t7.so $B/head.so $B/g_t6.so $B/g_t7.so $B/g_v2.so $B/g_v2t7.so" bash scripts/ab_configs.sh
