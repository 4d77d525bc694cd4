#!/bin/bash
# After scripts/gpu_profile_r6.sh on the GPU box: the records' raw CSVs, trimmed and gzipped by scripts/prof_commit.py,
# into $PACK/prof_NAME (what profiles/r06/prof/ holds), each checked to summarise to the same record; the raw session
# directories are then deleted so gpurun_out stays under the 64 MiB that gpurun copies back.
#   OUT=gpurun_out/r6prof PACK=gpurun_out/r6pack bash scripts/prof_pack.sh
set -o pipefail
OUT=${OUT:-gpurun_out/r6prof}; PACK=${PACK:-gpurun_out/r6pack}; mkdir -p $PACK
for rec in $OUT/counters_*.json; do
  name=$(basename $rec .json); name=${name#counters_}
  src=$OUT/prof_$name
  case $name in
    c4_*) extra="--keep-last k_ira_load:70 --decode k_ira_load,k_ira_vn,k_ira_cn,k_ira_out"
          sel="--decode-kernels k_ira_load,k_ira_vn,k_ira_cn,k_ira_out --chunks 35 --last 2";;
    c1_wifi648_minsum50) extra=""; sel="--kernel k_qc_ms_ph --last 11";;
    c1_wifi648_tanh50) extra=""; sel="--kernel k_qc_sp_st --last 11";;
    c2_*) extra=""; sel="--kernel k_qc_sp_rs --last 11";;
    c3_*) extra=""; sel="--kernel k_qc_qms_pk --last 11";;
  esac
  python3 scripts/prof_commit.py $src $PACK/prof_$name $extra || exit 1
  python3 scripts/counters_summary.py $PACK/prof_$name --name $name $sel > $PACK/check_$name.json || exit 1
  python3 -c "import json,sys; a=json.load(open('$rec')); b=json.load(open('$PACK/check_$name.json')); sys.exit(0 if a==b else 1)" \
    || { echo "packed copy of $name summarises differently"; exit 1; }
  cp $rec $PACK/
  rm -rf $src $PACK/check_$name.json
  echo "packed $name"
done
