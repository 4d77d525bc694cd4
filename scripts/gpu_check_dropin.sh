set -o pipefail
OUT=gpurun_out/dropin1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "decode_bits" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python bench.py --steps 11 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', round(d['value']/1e6,3), 'dropin', round(d['dropin_cw_per_s']/1e6,3), d['side']['dropin']['seconds'])"
