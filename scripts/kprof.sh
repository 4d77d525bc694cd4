#!/bin/bash
# Per-kernel profile of one bench configuration: kernel-trace stats, then one PMC pass per counter group, all
# summarised per kernel name (mean per dispatch) by scripts/kprof_summary.py.
#   OUT=gpurun_out/kp NAME=c4 ARGS="--code dvbs2_12 --batch 4096 --ebn0 1.5:1:1.5 --steps 2 --warmup 1" bash scripts/kprof.sh
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/kprof}; NAME=${NAME:-run}; D=$OUT/$NAME; mkdir -p $D
ARGS="$ARGS --no-dropin --no-legs --no-cpu-baseline"
GROUPS_=${GROUPS_:-"FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/ks -o run --output-format csv -- python3 bench.py $ARGS > $D/ks.json 2> $D/ks.err || { echo "kernel trace failed"; tail -5 $D/ks.err; exit 1; }
i=0
IFS='|' read -ra GS <<< "$GROUPS_"
for g in "${GS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $g --output-format csv -d $D/pmc$i -o run -- python3 bench.py $ARGS > $D/pmc$i.json 2> $D/pmc$i.err || { echo "pmc pass $i failed"; tail -5 $D/pmc$i.err; exit 1; }
done
python3 scripts/kprof_summary.py $D > $D/summary.txt && cat $D/summary.txt
