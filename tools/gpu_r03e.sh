#!/bin/bash
# Round-3: dynamics multi-pop A/B (parity + bench per variant), the graph-capture tests, and the
# bench's graph leg on the three workloads.  usage: bash tools/gpu_r03e.sh <tag> <variants...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r03e}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_rollout_gpu.py -x -q --timeout 300 --timeout-method thread > $O/rollout_tests.log 2>&1 || exit 10
for w in rollout sac-gru qmix; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --workload $w >> $O/graph_leg.jsonl 2>> $O/graph_leg.err || exit 11
done
CONFIGS="--batch 65536;--batch 4096;--trace poisson_for_loop_rate_500 --servers 8;--workload qmix" bash tools/gpu_ab.sh $TAG "$@"
