#!/bin/bash
# QMIX pair-kernel staging A/B (round 5): policy tests, then the configs[4] workloads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r05q2}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_policy.py tests/test_rollout_gpu.py -m gpu > $O/tests.txt 2>&1 || exit 11
bash tools/gpu_lib_ab.sh $TAG/qmix cur -- --workload qmix --steps 30 --warmup 5 || exit 12
bash tools/gpu_lib_ab.sh $TAG/qmix64 cur -- --workload qmix --servers 64 --steps 30 --warmup 5 || exit 13
