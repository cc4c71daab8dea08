#!/bin/bash
# Round-6: QMIX pair kernel with the first (hidden-pass) GRU weights requested after the staging
# loads (late: LBSIM_QMIX_PRIME_LATE=1) -- policy GPU tests on that build, then the qmix A/B.
#   usage: bash tools/gpu_r06za.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06za}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_late.so timeout -k 10 600 python -u -m pytest tests/test_fused_policy.py tests/test_rollout_gpu.py tests/test_multi_agent_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_late.log 2>&1 || exit 10
bash tools/gpu_lib_ab.sh $TAG/qmix cur late -- --workload qmix || exit 11
