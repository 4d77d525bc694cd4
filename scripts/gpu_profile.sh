#!/bin/bash
# One profiling session for one bench configuration, all on the same box and build:
#   1. bench.py (the number), 2. rocprofv3 --kernel-trace --stats (kernel durations),
#   3. PMC passes (kernel trace only, one counter group per pass): SQ issue/wait counters, LDS activity,
#      GRBM_GUI_ACTIVE (cycles), FETCH_SIZE, WRITE_SIZE (HBM traffic; separate TCC passes on gfx950),
#   4. scripts/counters_summary.py -> $OUT/counters_$NAME.json (per-launch means + derived fractions).
#     NAME=headline KERNEL=k_qc_ms ARGS="--steps 22 --warmup 3" bash scripts/gpu_profile.sh
set -o pipefail
OUT=${OUT:-gpurun_out}; mkdir -p $OUT; export TMPDIR=/tmp
NAME=${NAME:-headline}
KERNEL=${KERNEL:-k_qc_ms}
ARGS="${ARGS:-} --no-dropin"  # the drop-in / tanh-SP side measurements are not profiled
PARGS=${PARGS:---steps 4 --warmup 1}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
D=$OUT/prof_$NAME
mkdir -p $D
timeout -k 10 300 python3 bench.py $ARGS > $D/bench.json 2> $D/bench.err || { echo "bench $NAME failed"; tail -5 $D/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/ks -o run --output-format csv -- python3 bench.py $ARGS --no-cpu-baseline > $D/ks.json 2> $D/ks.err || { echo "kstats $NAME failed"; tail -5 $D/ks.err; exit 1; }
i=0
for grp in "$P1" "$P2" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $D/pmc$i -o run -- python3 bench.py $ARGS $PARGS --no-cpu-baseline > $D/pmc$i.json 2> $D/pmc$i.err || { echo "pmc pass $i ($NAME) failed"; tail -5 $D/pmc$i.err; exit 1; }
done
python3 scripts/counters_summary.py $D --name $NAME --kernel "$KERNEL" > $OUT/counters_$NAME.json && echo "counters_$NAME.json written"
python3 scripts/timed_launches.py $D --kernel "$KERNEL" > $D/timed.json 2>/dev/null || true
