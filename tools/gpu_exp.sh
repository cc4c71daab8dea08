#!/bin/bash
# Timing experiments: bench each prebuilt variant library .exp/lib_<name>.so (copied over the
# in-tree library of the GPU box's scratch copy) with the given bench args.
# usage: bash tools/gpu_exp.sh <tag> "<bench args>" [<name> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-exp}; ARGS=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/exp.jsonl
for n in "$@"; do
  cp .exp/lib_$n.so marllb_amd/liblbsim.so || exit 9
  echo "{\"variant\": \"$n\"}" >> $O/exp.jsonl
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $ARGS >> $O/exp.jsonl 2> $O/err_$n.log || exit 12
done
