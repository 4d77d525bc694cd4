#!/bin/bash
# One bench.py line per BASELINE.json config (the headline is configs[1]; the others document throughput
# of the parity-test configurations).  Each run has its own time limit; the chain stops on failure.
set -o pipefail
OUT=${OUT:-gpurun_out}; mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-dropin "$@" > $OUT/cfg_$name.json 2> $OUT/cfg_$name.err || { echo "$name failed"; tail -5 $OUT/cfg_$name.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$OUT/cfg_$name.json'));d['config']['name']='$name';print(json.dumps(d))" >> $OUT/bench_configs.jsonl
  python -c "import json;d=json.load(open('$OUT/cfg_$name.json'));print('$name', round(d['value']), 'cw/s', round(d['roofline']['launch_ms'],3), 'ms/launch', d['config']['kernel_path'])"
}
rm -f $OUT/bench_configs.jsonl
run c1_wifi648_minsum50 --steps 22
run c1_wifi648_tanh50 --steps 11 --algo tanh
run c1_wifi648_minsum50_generic --steps 11 --force-generic
run c2_wifi1944_tanh50_16qam --steps 11 --code wifi1944_56 --algo tanh --mod 16qam-ofdm --ebn0 4:0.5:9 --batch 32768
run c3_wifi1296_q5_20es --steps 11 --code wifi1296_23 --algo qminsum --iters 20 --early-stop --ebn0 0:0.5:5
run c3_wifi1296_q5_20_fixed --steps 11 --code wifi1296_23 --algo qminsum --iters 20
run c4_dvbs2_minsum50 --steps 5 --code dvbs2_12 --batch 4096 --ebn0 0:0.5:2
run c4_dvbs2_tanh50 --steps 3 --code dvbs2_12 --algo tanh --batch 4096 --ebn0 0:0.5:2
run c4_dvbs2s_minsum50 --steps 5 --code dvbs2s_12 --batch 4096 --ebn0 0:0.5:2
