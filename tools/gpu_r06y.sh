#!/bin/bash
# Round-6: the QMIX pair kernel with its obs rows loaded straight into LDS and the GRU's hidden pass
# first (LBSIM_QMIX_ASYNC_OBS=1 build "async") -- the policy / rollout / multi-agent GPU tests on
# that build, the qmix bench A/B against the shipped build, and its phase timeline.
#   usage: bash tools/gpu_r06y.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06y}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_async.so timeout -k 10 600 python -u -m pytest tests/test_fused_policy.py tests/test_rollout_gpu.py tests/test_multi_agent_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_async.log 2>&1 || exit 10
bash tools/gpu_lib_ab.sh $TAG/qmix cur async -- --workload qmix || exit 11
LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_asyncp.so timeout -k 10 300 python tools/policy_phases.py --workload qmix > $O/qmix_phases_async.jsonl 2> $O/phases.err || exit 12
