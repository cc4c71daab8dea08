#!/bin/bash
# Round-6: SAC at its new 32-env default (policy / rollout GPU tests), QMIX first GRU weights
# requested after the staging loads (qlate) against the shipped order, with phase timelines.
#   usage: bash tools/gpu_r06r.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06r}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_policy.py tests/test_rollout_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 10
bash tools/gpu_lib_ab.sh $TAG/qmix cur qlate -- --workload qmix || exit 11
for v in phases qlatep; do
  echo "== $v" >> $O/qmix_phases.jsonl
  LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_$v.so timeout -k 10 300 python tools/policy_phases.py --workload qmix >> $O/qmix_phases.jsonl 2>> $O/phases.err || exit 12
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 10 --workload sac-gru > $O/sac.json 2>> $O/bench.err || exit 13
