#!/bin/bash
# Same-box A/B over environment settings: for each ';'-separated bench argument list in CONFIGS
# and each ';'-separated VARS entry (an env assignment list, "-" = none), ROUNDS interleaved runs.
# usage: ROUNDS=2 CONFIGS="--batch 4096;--batch 65536" VARS="-;LBSIM_DYN_GROUP_LANES=16" bash tools/gpu_envab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-envab}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/ab.jsonl
IFS=';' read -ra CFG <<< "${CONFIGS:---batch 65536}"
IFS=';' read -ra VS <<< "${VARS:--}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${CFG[@]}"; do
    for v in "${VS[@]}"; do
      echo "{\"variant\": \"$v\", \"round\": $r, \"args\": \"$c\"}" >> $O/ab.jsonl
      if [ "$v" = "-" ]; then ev=""; else ev="$v"; fi
      env $ev timeout -k 10 240 python bench.py --no-cpu-baseline --steps ${STEPS:-30} --warmup 5 $c >> $O/ab.jsonl 2>> $O/err.log || exit 12
    done
  done
done
