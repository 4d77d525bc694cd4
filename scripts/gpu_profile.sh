#!/bin/bash
# One profiling session for one bench configuration, all on the same box and build:
#   1. bench.py (the number), 2. rocprofv3 --kernel-trace --stats (kernel durations),
#   3. PMC passes (kernel trace only, one counter group per pass): SQ issue/wait counters, LDS activity,
#      GRBM_GUI_ACTIVE (cycles), FETCH_SIZE, WRITE_SIZE (HBM traffic; separate TCC passes on gfx950),
#   4. scripts/counters_summary.py -> $OUT/counters_$NAME.json (per-launch MEANS + derived fractions).
# The kernel-trace and PMC passes run `--steps P --warmup P` with P = the number of Eb/N0 points of the
# grid: the BER pass, the warmup and the timed loop each decode once per point; the summary takes the timed
# loop's P launches (`--last P`), so the means cover the sweep evenly (the early-stop kernels' work depends
# on the point), after the clock ramp, and the trace and counters see the same launches.
#     NAME=headline KERNEL=k_qc_ms ARGS="" bash scripts/gpu_profile.sh
#     NAME=c4 DKERNELS=k_ira_load,k_ira_vn,k_ira_cn,k_ira_out CHUNKS=15 ARGS="--code dvbs2_12 --batch 4096 --ebn0 0:0.5:2" bash ...
set -o pipefail
OUT=${OUT:-gpurun_out}; mkdir -p $OUT; export TMPDIR=/tmp
NAME=${NAME:-headline}
ARGS="${ARGS:-} --no-dropin --no-legs"  # side measurements and the other configs' legs are not profiled
GRID=$(python3 -c "import sys; a=sys.argv[1:]; print(a[a.index('--ebn0')+1] if '--ebn0' in a else '0:0.5:5')" $ARGS)
P=$(python3 -c "import numpy as np,sys; lo,s,hi=map(float,sys.argv[1].split(':')); print(len(np.arange(lo,hi+1e-9,s)))" $GRID)
S=${STEPS:-$P}  # timed decodes (default: one per Eb/N0 point); the summary keeps the timed loop's S launches
PARGS="--steps $S --warmup $S --no-cpu-baseline"
if [ -n "$DKERNELS" ]; then SEL="--decode-kernels $DKERNELS --chunks ${CHUNKS:-1}"; else SEL="--kernel ${KERNEL:-k_qc_ms}"; fi
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
D=$OUT/prof_$NAME
mkdir -p $D
echo "profile $NAME: $ARGS ($P points)"
timeout -k 10 300 python3 bench.py $ARGS > $D/bench.json 2> $D/bench.err || { echo "bench $NAME failed"; tail -5 $D/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/ks -o run --output-format csv -- python3 bench.py $ARGS $PARGS > $D/ks.json 2> $D/ks.err || { echo "kstats $NAME failed"; tail -5 $D/ks.err; exit 1; }
i=0
for grp in "$P1" "$P2" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $D/pmc$i -o run -- python3 bench.py $ARGS $PARGS > $D/pmc$i.json 2> $D/pmc$i.err || { echo "pmc pass $i ($NAME) failed"; tail -5 $D/pmc$i.err; exit 1; }
  echo "  pmc pass $i done"
done
python3 scripts/counters_summary.py $D --name $NAME $SEL --last $S > $OUT/counters_$NAME.json && echo "counters_$NAME.json written"
