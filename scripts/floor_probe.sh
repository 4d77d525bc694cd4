#!/bin/bash
# Per-launch floor (LLR load, quantize, output) vs per-iteration cost of the register kernels: bench launches at a
# few iteration counts; the intercept of launch time over iterations is the floor.
set -o pipefail
export TMPDIR=/tmp
for c in "c1|" "c3|--code wifi1296_23 --algo qminsum" "t1|--algo tanh --clamp 10"; do
  n=${c%%|*}; a=${c#*|}
  for it in 1 2 5 10; do
    timeout -k 10 120 python bench.py $a --iters $it --ebn0 2:0.5:2 --no-legs --no-dropin --no-cpu-baseline --steps 20 --warmup 3 > /tmp/o.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('/tmp/o.json'));print('$n', $it, 'iters', round(d['roofline']['launch_ms'],4), 'ms')"
  done
done
