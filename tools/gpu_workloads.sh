#!/bin/bash
# Every BASELINE workload line, the async / late-episode legs, the single-env latency and the
# 4k-512k sweep (tools/gpu_round.sh steps 4-5 without the tests).  usage: bash tools/gpu_workloads.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-workloads}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/workloads.jsonl
for a in "--batch 4096" "--batch 4096 --servers 8" "--trace poisson_for_loop_rate_500 --servers 8" "--workload sac-gru" "--workload qmix" "--workload qmix --servers 64"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $a >> $O/workloads.jsonl 2>> $O/workloads.err || exit 14
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --async-groups 2 --late-episode 1000,5000 > $O/async_late.json 2>> $O/workloads.err || exit 15
timeout -k 10 300 python tools/single_env_latency.py --steps 2000 > $O/single_env_latency.json 2>> $O/workloads.err || exit 16
bash tools/gpu_sweep.sh $TAG --no-graph || exit 17
