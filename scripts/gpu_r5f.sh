# round 5 session f: zero-LLR scan + forked a == 1 pass — parity (scale, graph capture), config [2] A/B and trace
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5f}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_zero_pass.py tests/test_gpu_parity.py tests/test_gpu_config2.py tests/test_gpu_soft_parity.py tests/test_gpu_bench_legs.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT CONFIGS="c2|--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 4:0.5:9 --no-legs --steps 11 --warmup 3;t648|--code wifi648_12 --algo tanh --iters 50 --clamp 20 --batch 65536 --no-legs" \
  VARIANTS="build_variants/fix0_all.so build_variants/cur.so build_variants/fix0_all.so build_variants/cur.so" bash scripts/ab_configs.sh || exit 1
C2="--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 6:1:6 --steps 3 --warmup 1 --no-dropin --no-legs --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2_cur -o run --output-format csv -- python3 bench.py $C2 > $OUT/c2_cur.json 2> $OUT/c2_cur.err || { tail -5 $OUT/c2_cur.err; exit 1; }
python3 - $OUT/c2_cur/run_kernel_trace.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sp_rs" in r["Kernel_Name"] or "zero_scan" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
for r in rows[-9:]:
    print(f'{r["Kernel_Name"][:48]:48s} start {(int(r["Start_Timestamp"]) - t0) / 1e3:10.1f} us  dur {(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:8.1f} us')
PY
