#!/bin/bash
# One bench line per BASELINE config workload, then the batch sweep (4k -> 512k at S = 4 and 8).
# usage: bash tools/gpu_workloads.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-workloads}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/workloads.jsonl
for a in "--batch 4096" "--trace poisson_for_loop_rate_500 --servers 8" "--workload sac-gru" "--workload qmix" "--workload qmix --servers 64"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $a >> $O/workloads.jsonl 2>> $O/workload_err.log || exit 21
done
bash tools/gpu_sweep.sh $TAG
