#!/bin/bash
# Simulator + rollout GPU tests, then the three workloads with their graph legs.  usage: bash tools/gpu_graph_legs.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-grst}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_env_gpu.py tests/test_rollout_gpu.py tests/test_multi_agent_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 10
for w in rollout sac-gru qmix; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --workload $w >> $O/graph.jsonl 2>> $O/err.log || exit 11
done
