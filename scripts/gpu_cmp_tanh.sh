#!/bin/bash
# Bitwise A/B of build_variants/base.so against the in-tree library (scripts/cmp_libs.py), GPU tests, tanh-SP config benches.
set -o pipefail
mkdir -p gpurun_out
LDPC_LIB=$PWD/build_variants/base.so timeout -k 10 300 python scripts/cmp_libs.py gpurun_out/cmp_a.npz > gpurun_out/cmp_a.log 2>&1 || { echo cmp_a failed; tail gpurun_out/cmp_a.log; exit 1; }
timeout -k 10 300 python scripts/cmp_libs.py gpurun_out/cmp_b.npz > gpurun_out/cmp_b.log 2>&1 || { echo cmp_b failed; tail gpurun_out/cmp_b.log; exit 1; }
python scripts/cmp_libs.py --compare gpurun_out/cmp_a.npz gpurun_out/cmp_b.npz | tee gpurun_out/cmp.log; rm -f gpurun_out/cmp_?.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
for a in "t648 --steps 11 --algo tanh" "t1944 --steps 11 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768" "tdvb --steps 3 --code dvbs2s_12 --algo tanh --batch 4096 --ebn0 0:0.5:2"; do
  set -- $a; n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/t_$n.json 2> gpurun_out/t_$n.err || { echo "$n failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/t_$n.json'));print('$n', round(d['value']), 'cw/s', round(d['roofline']['launch_ms'],3), 'ms', d['config']['kernel_path'], d['ber']['coded_bler'][:6])"
done
