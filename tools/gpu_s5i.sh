#!/bin/bash
# Chained profiler events: tests + smoke + bench + kernel trace (gpu_check.sh), two more bench runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-s5i}
O=$R/gpurun_out/$TAG
bash $R/tools/gpu_check.sh $TAG || exit $?
cd $R
: > $O/ab.jsonl
for rep in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline >> $O/ab.jsonl 2>> $O/ab.err || exit 11
done
