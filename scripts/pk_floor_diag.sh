# Prices config [3]'s per-launch floor with diagnostic builds of the packed kernel (QC_PK_DIAG, wrong results):
# pkD1 = no bit stores, pkD2 = no LLR loads, vs the shipped build.  Build first (CPU):
#   cp ldpc-sims_amd/ldpc_amd/libldpc_hip.so build_variants/base.so
#   bash scripts/mkvariant.sh pkD1 qc_pk.hip -DQC_PK_DIAG=1; bash scripts/mkvariant.sh pkD2 qc_pk.hip -DQC_PK_DIAG=2
set -o pipefail
export TMPDIR=/tmp
B=build_variants
OUT=gpurun_out/pkdiag CONFIGS="es1|--code wifi1296_23 --algo qminsum --iters 1 --early-stop --ebn0 5:0.5:5 --no-legs --steps 20;fx1|--code wifi1296_23 --algo qminsum --iters 1 --ebn0 5:0.5:5 --no-legs --steps 20" VARIANTS="$B/base.so $B/pkD1.so $B/pkD2.so $B/base.so $B/pkD1.so $B/pkD2.so" bash scripts/ab_configs.sh
