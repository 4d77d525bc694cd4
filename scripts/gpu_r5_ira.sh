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
# config [2] soft-parity trace: shipped build and the correctly-rounded diagnostic variants (DS_CR)
timeout -k 10 300 python scripts/trace_config2.py --label shipped > $OUT/trace_c2_shipped.json 2> $OUT/trace_c2_shipped.err || { tail -20 $OUT/trace_c2_shipped.err; exit 1; }
for v in 1 2 4 7; do
  LDPC_LIB=$PWD/build_variants/cr$v.so timeout -k 10 300 python scripts/trace_config2.py --label cr$v > $OUT/trace_c2_cr$v.json 2> $OUT/trace_c2_cr$v.err || { tail -20 $OUT/trace_c2_cr$v.err; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5_ira/trace_c2_*.json")):
    d = json.load(open(f))
    print(d["label"], "decoded", d["decoded"], "late", d["converged_after_40"], "gpu/f64 by40 %.2e after40 %.2e" % (d["gpu_vs_f64_max_by_40"], d["gpu_vs_f64_max_after_40"]),
          "oracle/f64 after40 %.2e" % d["oracle_vs_f64_max_after_40"], "rows==oracle", d["gpu_eq_oracle_bitwise_rows"], "entries==", round(d["gpu_eq_oracle_bitwise_entries_frac"], 5),
          "first_ne", [r["first_gpu_ne_oracle_iter"] for r in d["rows"]])
PY
for v in shipped 7; do
  lib=""; [ $v = 7 ] && lib=$PWD/build_variants/cr7.so
  LDPC_LIB=$lib timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --legs config2 > $OUT/c2_$v.json 2> $OUT/c2_$v.err || { tail -20 $OUT/c2_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c2_$v.json'));l=d['side']['configs']['config2'];print('config2 $v', round(l['value']/1e6,3), 'M cw/s', round(l['ms_per_launch'],3), 'ms')"
done
