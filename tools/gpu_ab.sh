#!/bin/bash
# Same-box A/B over several bench configurations: every prebuilt variant library
# expl/lib_<name>.so (copied over the in-tree library of the GPU box's scratch copy) is benched on
# every configuration in CONFIGS (';'-separated bench argument lists), interleaved over ROUNDS
# rounds so drift between rounds does not favour one variant.
# usage: ROUNDS=2 CONFIGS="--batch 65536;--batch 131072" bash tools/gpu_ab.sh <tag> <name> [<name> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-ab}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
cp marllb_amd/liblbsim.so $O/lib_orig.so
: > $O/ab.jsonl
IFS=';' read -ra CFG <<< "${CONFIGS:---batch 65536}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${CFG[@]}"; do
    for n in "$@"; do
      cp expl/lib_$n.so marllb_amd/liblbsim.so || exit 9
      echo "{\"variant\": \"$n\", \"round\": $r, \"args\": \"$c\"}" >> $O/ab.jsonl
      timeout -k 10 240 python bench.py --no-cpu-baseline --steps ${STEPS:-30} --warmup 5 $c >> $O/ab.jsonl 2> $O/err_$n.log || exit 12
    done
  done
done
cp $O/lib_orig.so marllb_amd/liblbsim.so
