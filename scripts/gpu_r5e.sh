# round 5 session e: block-boundary parity test, IRA defaults (tpw 4, 256 MB) profile, config [2] pass split trace
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5e}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_cn_blocks.py tests/test_gpu_ira.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT/kp NAME=c4 ARGS="--code dvbs2_12 --batch 4096 --ebn0 1.5:1:1.5 --steps 2 --warmup 1" bash scripts/kprof.sh > /dev/null || exit 1
head -4 $OUT/kp/c4/summary.txt | cut -c1-250
C2="--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 6:1:6 --steps 3 --warmup 1 --no-dropin --no-legs --no-cpu-baseline"
for v in cur c2_fix0; do
  LDPC_LIB=$PWD/build_variants/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2_$v -o run --output-format csv -- python3 bench.py $C2 > $OUT/c2_$v.json 2> $OUT/c2_$v.err || { tail -5 $OUT/c2_$v.err; exit 1; }
  python3 - $OUT/c2_$v/run_kernel_trace.csv $v <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
t = collections.defaultdict(list)
for r in rows:
    t[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(t.items(), key=lambda kv: -sum(kv[1]))[:6]:
    print(sys.argv[2], f"{k:60s} n={len(v):4d} mean={sum(v)/len(v):9.2f} us")
PY
done
