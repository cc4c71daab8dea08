#!/bin/bash
# QMIX policy kernel A/B: policy parity tests on this tree, then --workload qmix interleaved
# between this tree's library (base) and variant libraries.  usage: bash tools/gpu_qmix_ab.sh <tag> <variant...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-qab}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_fused_policy.py tests/test_rollout_gpu.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || exit 10
PARITY=0 ROUNDS=3 CONFIGS="--workload qmix" bash tools/gpu_ab.sh $TAG base "$@"
