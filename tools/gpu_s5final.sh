#!/bin/bash
# Session-5 round-end pass: gpu_final.sh (tests, smoke, bench, kernel trace, PMC, workloads), then
# the async env-group measurements (bench.py --async-groups) at 65536 x 4 and configs[2].
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-final}
O=$R/gpurun_out/$TAG
bash $R/tools/gpu_final.sh $TAG || exit $?
cd $R
: > $O/async_groups.jsonl
for g in 2 4; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --async-groups $g >> $O/async_groups.jsonl 2>> $O/async_err.log || exit 40
  timeout -k 10 180 python bench.py --no-cpu-baseline --servers 8 --trace poisson_for_loop_rate_500 --async-groups $g >> $O/async_groups.jsonl 2>> $O/async_err.log || exit 41
done
