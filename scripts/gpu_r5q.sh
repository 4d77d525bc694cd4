# round 5 session q: IRA streams x budget after the parity fusion
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5q}; mkdir -p $OUT
C4="--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --no-legs"
for v in 2:200 3:200 2:240 3:240 2:160 4:240 2:200; do
  ns=${v%%:*}; mb=${v#*:}
  LDPC_IRA_STREAMS=$ns LDPC_IRA_BUDGET_MB=$mb timeout -k 10 300 python bench.py $C4 > $OUT/c4_s${ns}_b$mb.json 2> $OUT/c4_s${ns}_b$mb.err || { tail -20 $OUT/c4_s${ns}_b$mb.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_s${ns}_b$mb.json'));r=d['roofline'];print('streams $ns budget $mb', round(d['value']), 'cw/s', round(r['launch_ms'],2), 'ms')"
done
