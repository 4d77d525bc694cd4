# (D, S) join with fma (DS_JOIN_FMA=1, join1) vs two products and an add (join0): tanh-SP configs
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/join \
CONFIGS="c1tanh|--code wifi648_12 --algo tanh --iters 50 --clamp 10 --no-legs --steps 11 --warmup 3;c2|--code wifi1944_56 --algo tanh --iters 50 --clamp 20 --batch 32768 --mod 16qam-ofdm --ebn0 4:0.5:9 --no-legs --steps 11 --warmup 3" \
VARIANTS="build_variants/join0.so build_variants/join1.so build_variants/join0.so build_variants/join1.so" bash scripts/ab_configs.sh
