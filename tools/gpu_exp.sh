#!/bin/bash
# Same-box A/B timing: bench each prebuilt variant library expl/lib_<name>.so (copied over the
# in-tree library of the GPU box's scratch copy), interleaved over ROUNDS rounds so drift between
# rounds does not favour one variant.
# usage: ROUNDS=2 bash tools/gpu_exp.sh <tag> "<bench args>" [<name> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-exp}; ARGS=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
cp marllb_amd/liblbsim.so $O/lib_orig.so
: > $O/exp.jsonl
for r in $(seq 1 ${ROUNDS:-2}); do
  for n in "$@"; do
    cp expl/lib_$n.so marllb_amd/liblbsim.so || exit 9
    echo "{\"variant\": \"$n\", \"round\": $r}" >> $O/exp.jsonl
    timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $ARGS >> $O/exp.jsonl 2> $O/err_$n.log || exit 12
  done
done
cp $O/lib_orig.so marllb_amd/liblbsim.so
