set -o pipefail
export TMPDIR=/tmp
for a in "--iters 1 --early-stop --ebn0 5:0.5:5" "--iters 1 --ebn0 5:0.5:5" "--iters 2 --ebn0 5:0.5:5" "--iters 20 --early-stop --ebn0 5:0.5:5" "--iters 20 --ebn0 5:0.5:5" "--iters 20 --early-stop --ebn0 0:0.5:0" "--iters 4 --ebn0 5:0.5:5"; do
  timeout -k 10 120 python bench.py --code wifi1296_23 --algo qminsum --no-legs --no-dropin --no-cpu-baseline --steps 10 --warmup 2 $a > /tmp/o.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('/tmp/o.json'));print('$a', round(d['roofline']['launch_ms'],4), 'ms')"
done
