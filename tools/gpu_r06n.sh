#!/bin/bash
# Round-6: the policy kernels with every staging load in flight together -- their GPU tests, the
# phase timelines (LBSIM_EXP_PHASES build) and the sac-gru / qmix bench lines.
#   usage: bash tools/gpu_r06n.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06n}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_policy.py tests/test_rollout_gpu.py tests/test_multi_agent_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 10
for w in qmix sac-gru; do
  LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_phases.so timeout -k 10 300 python tools/policy_phases.py --workload $w >> $O/phases.jsonl 2>> $O/phases.err || exit 11
done
for rep in 1 2; do
  for w in sac-gru qmix; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 10 --workload $w >> $O/policy.jsonl 2>> $O/bench.err || exit 12
  done
done
