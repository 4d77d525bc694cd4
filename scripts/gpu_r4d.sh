#!/bin/bash
# Round 4 session d: headline priority refinement A/B, full GPU suite, bench line, every counter record re-profiled.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
LDPC_LIB=$PWD/build_variants/phP3.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x --timeout 250 -k "minsum_bit_exact" > $O/check_phP3.log 2>&1 || { echo "phP3 FAILED parity"; exit 1; }
OUT=$O CONFIGS="c1|--no-legs --steps 22" VARIANTS="build_variants/base.so build_variants/phP3.so build_variants/base.so build_variants/phP3.so build_variants/base.so build_variants/phP3.so" bash scripts/ab_configs.sh || exit 1
LDPC_PARITY_LOG=$O/soft_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench.json'));print('bench', round(d['value']/1e6,3), d['roofline']['bound'], round(d['roofline']['frac'],3), 'tanh', round(d['side']['gpu_tanh_sp']['cw_per_s']/1e6,3), 'dropin', round(d['dropin_cw_per_s']/1e6,3))
for k, l in d['side']['configs'].items(): print(k, round(l['value']/1e6, 4), 'M cw/s', l['roofline']['bound'], round(l['roofline']['frac'],3))"
OUT=$O/prof bash scripts/gpu_profile_r4.sh
