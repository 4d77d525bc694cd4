# tanh-SP (648,1/2) register kernel tunables after the fma join (k_qc_sp_st; bench --algo tanh --clamp 10)
set -o pipefail
export TMPDIR=/tmp
B=build_variants
OUT=gpurun_out/sp2 CONFIGS="c1tanh|--code wifi648_12 --algo tanh --iters 50 --clamp 10 --no-legs --steps 11 --warmup 3" \
VARIANTS="$B/head.so $B/sp_ss2.so $B/sp_gla.so $B/sp_p0.so $B/sp_p1.so $B/head.so $B/sp_ss2.so $B/sp_gla.so $B/sp_p0.so $B/sp_p1.so" bash scripts/ab_configs.sh
