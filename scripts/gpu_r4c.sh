#!/bin/bash
# Round 4 session c: full GPU suite (soft-parity log), smoke, the GPU soft-output trace, the bench line, and a
# counter profile of config [2]'s resident kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
LDPC_PARITY_LOG=$O/soft_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
timeout -k 10 300 python scripts/trace_failure_gpu.py || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench.json'));print('bench', round(d['value']/1e6,3), d['roofline']['bound'], round(d['roofline']['frac'],3), 'tanh', round(d['side']['gpu_tanh_sp']['cw_per_s']/1e6,3))
for k, l in d['side']['configs'].items(): print(k, round(l['value']/1e6, 4), 'M cw/s', l['roofline']['bound'], round(l['roofline']['frac'],3), l['roofline']['counters'])"
OUT=$O NAME=c2_wifi1944_tanh50_16qam KERNEL=k_qc_sp_rs ARGS="--code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" bash scripts/gpu_profile.sh
