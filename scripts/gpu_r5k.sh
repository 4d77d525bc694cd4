# round 5 session k: IRA chunks on 1-4 streams — parity and A/B
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5k}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ira.py tests/test_gpu_zero_pass.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
C4="--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --no-legs"
for v in 2:256 3:256 4:256 3:200 4:200 2:200 1:256 3:256; do
  ns=${v%%:*}; mb=${v#*:}
  LDPC_IRA_STREAMS=$ns LDPC_IRA_BUDGET_MB=$mb timeout -k 10 300 python bench.py $C4 > $OUT/c4_s${ns}_b$mb.json 2> $OUT/c4_s${ns}_b$mb.err || { tail -20 $OUT/c4_s${ns}_b$mb.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_s${ns}_b$mb.json'));r=d['roofline'];print('streams $ns budget $mb', round(d['value']), 'cw/s', round(r['launch_ms'],2), 'ms', d['config']['kernel_path'])"
done
