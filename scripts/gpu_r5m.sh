# round 5 session m: IRA tasks per workgroup tuned per kernel (VN, CN)
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5m}; mkdir -p $OUT
C4="--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --no-legs"
for v in 4:4 2:4 3:4 6:4 8:4 4:2 4:6 4:8 4:4; do
  vn=${v%%:*}; cn=${v#*:}
  LDPC_IRA_TPW_VN=$vn LDPC_IRA_TPW=$cn timeout -k 10 300 python bench.py $C4 > $OUT/c4_v${vn}_c$cn.json 2> $OUT/c4_v${vn}_c$cn.err || { tail -20 $OUT/c4_v${vn}_c$cn.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_v${vn}_c$cn.json'));r=d['roofline'];print('vn $vn cn $cn', round(d['value']), 'cw/s', round(r['launch_ms'],2), 'ms')"
done
