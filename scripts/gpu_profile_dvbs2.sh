set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/dvb1; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/ks -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-dropin --code dvbs2_12 --batch 4096 --steps 3 --warmup 1 --ebn0 0:0.5:2 > $D/ks.json 2> $D/ks.err || { echo "ks failed"; tail -5 $D/ks.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_f -o run -- python3 bench.py --no-cpu-baseline --no-dropin --code dvbs2_12 --batch 4096 --steps 2 --warmup 0 --ebn0 0:0.5:2 > $D/f.json 2> $D/f.err || { echo "fetch failed"; tail -5 $D/f.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_w -o run -- python3 bench.py --no-cpu-baseline --no-dropin --code dvbs2_12 --batch 4096 --steps 2 --warmup 0 --ebn0 0:0.5:2 > $D/w.json 2> $D/w.err || { echo "write failed"; tail -5 $D/w.err; exit 1; }
echo done
