#!/bin/bash
# tests + smoke; headline A/B (16 / 13 / 12 envs per dynamics wave, r04f); the default bench line
# (graph leg: 5 steps per graph, next-step auto-reset); small-batch workloads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04l}
O=$R/gpurun_out/$TAG
bash $R/tools/gpu_tests.sh $TAG || exit $?
bash $R/tools/gpu_lib_ab.sh $TAG cur cur:LBSIM_DYN_EPW=13 cur:LBSIM_DYN_EPW=12 r04f || exit $?
cd $R
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 12
: > $O/workloads.jsonl
for a in "--batch 4096" "--batch 4096 --servers 8"; do
  echo "== $a" >> $O/workloads.jsonl
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 $a >> $O/workloads.jsonl 2>> $O/workloads.err || exit 14
done
