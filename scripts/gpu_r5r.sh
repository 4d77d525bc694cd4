# round 5 session r: IRA check rows per workgroup after the parity fusion
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5r}; mkdir -p $OUT
C4="--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --no-legs"
for v in 6 9 10 15 5 6; do
  cn=$v
  LDPC_IRA_TPW_CN=$cn timeout -k 10 300 python bench.py $C4 > $OUT/c4_cn$cn.json 2> $OUT/c4_cn$cn.err || { tail -20 $OUT/c4_cn$cn.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_cn$cn.json'));r=d['roofline'];print('cn $cn', round(d['value']), 'cw/s', round(r['launch_ms'],2), 'ms')"
done
