# round 5 session d: zero-LLR list (second pass walks a list), IRA balanced chunks + tasks-per-workgroup/budget sweep
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5d}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_config2.py tests/test_gpu_ira.py tests/test_gpu_soft_parity.py -k "zero or config2 or resident or kernels_agree or tanh or ira or sp or soft" > $OUT/pytest.log 2>&1; rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
C4="--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --no-legs"
for v in 2:200 4:200 2:240 3:240 4:240 2:256 4:256; do
  tpw=${v%%:*}; mb=${v#*:}
  LDPC_IRA_TPW=$tpw LDPC_IRA_BUDGET_MB=$mb timeout -k 10 300 python bench.py $C4 > $OUT/c4_t${tpw}_b$mb.json 2> $OUT/c4_t${tpw}_b$mb.err || { tail -20 $OUT/c4_t${tpw}_b$mb.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_t${tpw}_b$mb.json'));r=d['roofline'];print('tpw $tpw budget $mb', round(d['value']), 'cw/s', round(r['launch_ms'],2), 'ms', d['config']['kernel_path'])"
done
OUT=$OUT CONFIGS="c2|--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 4:0.5:9 --no-legs --steps 11 --warmup 3" \
  VARIANTS="build_variants/c2_fix0.so build_variants/cur.so build_variants/c2_fix0.so build_variants/cur.so" bash scripts/ab_configs.sh || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --legs config2 > $OUT/legs.json 2> $OUT/legs.err || { tail -20 $OUT/legs.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/legs.json'));[print(k, round(l['value']/1e6,3), 'M cw/s', round(l['ms_per_launch'],3), 'ms') for k,l in d['side']['configs'].items()]"
