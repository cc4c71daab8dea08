#!/bin/bash
# tests + smoke, library A/B at the headline, then the small-batch and wide-env workloads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04h}
O=$R/gpurun_out/$TAG
bash $R/tools/gpu_tests.sh $TAG || exit $?
bash $R/tools/gpu_lib_ab.sh $TAG cur r04f || exit $?
cd $R
: > $O/workloads.jsonl
for a in "--batch 4096" "--batch 4096 --servers 8" "--workload qmix --servers 64" "--workload qmix"; do
  echo "== $a" >> $O/workloads.jsonl
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 $a >> $O/workloads.jsonl 2>> $O/workloads.err || exit 14
done
