#!/bin/bash
# GPU session: full GPU tests (soft-parity / overlay log), smoke, the bench line, per-config lines.
#   OUT=gpurun_out/<name> bash scripts/gpu_session.sh
set -o pipefail
OUT=${OUT:-gpurun_out/session}
mkdir -p $OUT
export TMPDIR=/tmp
rm -f $OUT/soft_parity.jsonl
LDPC_PARITY_LOG=$OUT/soft_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
python -c "
import json;d=json.load(open('$OUT/bench.json'));print('bench', round(d['value']/1e6,3), d['roofline']['bound'], round(d['roofline']['frac'],3), 'dropin', round(d['dropin_cw_per_s']/1e6,3), 'tanh', round(d['side']['gpu_tanh_sp']['cw_per_s']/1e6,3))
for k, l in d['side']['configs'].items(): print(k, l['config']['workload'], round(l['value']/1e6, 4), 'M cw/s', l['roofline']['bound'], l['roofline']['frac'], l['roofline']['counters'])"
