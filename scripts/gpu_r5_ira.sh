# IRA (DVB-S2) kernels: parity tests, then config [4] bench A/B against the generic kernels
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5_ira}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_ira.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ira.log 2>&1 || { tail -40 $OUT/pytest_ira.log; exit 1; }
tail -3 $OUT/pytest_ira.log
C4="--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --no-legs"
for v in ira generic; do
  if [ $v = generic ]; then export LDPC_NO_IRA=1; else unset LDPC_NO_IRA; fi
  timeout -k 10 300 python bench.py $C4 > $OUT/c4_$v.json 2> $OUT/c4_$v.err || { tail -20 $OUT/c4_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_$v.json'));r=d['roofline'];print('$v', round(d['value']), 'cw/s', round(r['launch_ms'],2), 'ms', d['config']['kernel_path'], r['bound'], round(r['frac'],3), d['ber']['coded_bler'])"
done
unset LDPC_NO_IRA
for b in 0 100 400; do
  LDPC_IRA_BUDGET_MB=$b timeout -k 10 300 python bench.py $C4 > $OUT/c4_b$b.json 2> $OUT/c4_b$b.err || { tail -20 $OUT/c4_b$b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_b$b.json'));r=d['roofline'];print('budget $b', round(d['value']), 'cw/s', round(r['launch_ms'],2), 'ms')"
done
