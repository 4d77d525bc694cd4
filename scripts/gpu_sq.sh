#!/bin/bash
# SQ counters for the decode kernel (one rocprofv3 pass per counter group; kernel trace only).
#   COUNTERS="A B C|D E" bash scripts/gpu_sq.sh      ('|' separates passes)
set -o pipefail
OUT=${OUT:-gpurun_out}; mkdir -p $OUT; export TMPDIR=/tmp
ARGS=${ARGS:---steps 4 --warmup 1 --no-cpu-baseline}
KERNEL=${KERNEL:-k_qc_ms}
COUNTERS=${COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY|SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA"}
i=0
IFS='|' read -ra PASSES <<< "$COUNTERS"
for grp in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq$i -o run -- python3 bench.py $ARGS > $OUT/sq$i.json 2> $OUT/sq$i.err || { echo "pass $i failed"; tail -5 $OUT/sq$i.err; exit 1; }
done
KERNEL=$KERNEL OUT=$OUT python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(list)
for f in glob.glob(os.environ["OUT"] + "/sq*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if os.environ["KERNEL"] in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:32s} {sum(v)/len(v):.4g}")
PY
