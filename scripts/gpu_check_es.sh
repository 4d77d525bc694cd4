set -o pipefail
OUT=gpurun_out/es1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for a in "sl --steps 11" "gen --steps 11 --force-generic"; do set -- $a; n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-dropin --code wifi1944_56 --algo tanh --early-stop --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { echo "bench $n failed"; tail -5 $OUT/b_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_$n.json'));print('$n', round(d['value']/1e6,3), 'Mcw/s', d['config']['kernel_path'], [round(x,4) for x in d['ber']['coded_bler']])"
done
