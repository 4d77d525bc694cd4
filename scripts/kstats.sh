#!/bin/bash
# rocprofv3 kernel stats for one bench config: kstats.sh NAME [bench args...]; prints the top kernels.
set -o pipefail
OUT=${OUT:-gpurun_out}; mkdir -p $OUT
export TMPDIR=/tmp
name=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks_$name -o run --output-format csv -- python3 bench.py --no-cpu-baseline --warmup 1 "$@" > $OUT/ks_$name.json 2> $OUT/ks_$name.err || { echo "kstats $name failed"; tail -5 $OUT/ks_$name.err; exit 1; }
f=$(find $OUT/ks_$name -name "*kernel_stats.csv" | head -1)
python3 - "$f" "$name" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("==", sys.argv[2])
for r in rows[:6]:
    print(f"  {r['Name'][:90]:90s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
PY
