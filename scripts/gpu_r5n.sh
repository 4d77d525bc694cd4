# round 5 session n: IRA parity (per-kernel tasks per workgroup, host pointers over two streams) and the config [4] leg
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5n}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_ira.py tests/test_gpu_bench_legs.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --legs config4 > $OUT/legs.json 2> $OUT/legs.err || { tail -20 $OUT/legs.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/legs.json'));[print(k, round(l['value']), 'cw/s', round(l['ms_per_launch'],3), 'ms', l['roofline']['bound'], round(l['roofline']['frac'],3), l['roofline']['counters']) for k,l in d['side']['configs'].items()]"
