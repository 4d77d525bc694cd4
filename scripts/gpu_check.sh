# full GPU check of the in-tree build: -m gpu suite (asserting FAILURE_BOUNDS), smoke(), default bench line
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/check}; mkdir -p $OUT
rm -f $OUT/soft_parity.jsonl
LDPC_PARITY_LOG=$PWD/$OUT/soft_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -10 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -10 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print('headline', round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms', 'roofline', d['roofline']['bound'], round(d['roofline']['frac'],3))
s=d['side']; print('tanh', round(s['gpu_tanh_sp']['cw_per_s']/1e6,2), 'M')
for k,v in s.get('configs',{}).items(): print(k, round(v['value']/1e6,3), 'M', round(v['ms_per_step'],3), 'ms', v['roofline']['bound'], round(v['roofline']['frac'],3))"
