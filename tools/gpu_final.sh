#!/bin/bash
# Round-end GPU pass: parity tests + smoke + headline bench + rocprofv3 kernel trace (gpu_check.sh),
# PMC traffic / SQ passes (gpu_pmc.sh), then one bench line per BASELINE config workload.
# usage: bash tools/gpu_final.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-final}
O=$R/gpurun_out/$TAG
cd $R
bash tools/gpu_check.sh $TAG || exit $?
bash tools/gpu_pmc.sh ${TAG}_pmc || exit 20
cd $R
: > $O/workloads.jsonl
for a in "--batch 4096" "--trace poisson_for_loop_rate_500 --servers 8" "--workload sac-gru" "--workload qmix"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $a >> $O/workloads.jsonl 2> $O/workload_err.log || exit 21
done
