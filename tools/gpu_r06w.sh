#!/bin/bash
# Round-6: the 32-env SAC tile with its heads' partials halved (4 workgroups per CU instead of 3)
# against the previous form (m0: LBSIM_SAC_SPLIT_M=0) -- policy / rollout GPU tests, then the
# sac-gru bench A/B.   usage: bash tools/gpu_r06w.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06w}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_policy.py tests/test_rollout_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 10
bash tools/gpu_lib_ab.sh $TAG/sac m0 cur -- --workload sac-gru || exit 11
