# round 5 session i: IRA tasks side by side per workgroup (TPP) — parity and A/B with tasks one after the other (TPW)
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5i}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ira.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
C4="--code dvbs2_12 --iters 50 --batch 4096 --ebn0 0:0.5:2 --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --no-legs"
for v in 1:4 2:2 2:4 2:1 1:3 2:3 1:4; do
  tpp=${v%%:*}; tpw=${v#*:}
  LDPC_IRA_TPP=$tpp LDPC_IRA_TPW=$tpw timeout -k 10 300 python bench.py $C4 > $OUT/c4_p${tpp}_t$tpw.json 2> $OUT/c4_p${tpp}_t$tpw.err || { tail -20 $OUT/c4_p${tpp}_t$tpw.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/c4_p${tpp}_t$tpw.json'));r=d['roofline'];print('tpp $tpp tpw $tpw', round(d['value']), 'cw/s', round(r['launch_ms'],2), 'ms', d['config']['kernel_path'])"
done
