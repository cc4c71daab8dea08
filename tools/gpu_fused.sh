#!/bin/bash
# Fused policy kernels: GPU tests (fused, policies, rollouts), bench lines of configs[3] / [4] with
# the env tile swept (LBSIM_FUSED_MT), rocprofv3 kernel stats of both workloads.
# usage: bash tools/gpu_fused.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-fused}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_fused_policy.py tests/test_policies.py tests/test_rollout_gpu.py > $O/pytest.log 2>&1 || exit 10
: > $O/bench.jsonl
for mt in 0 1 2 4; do
  for w in qmix sac-gru; do
    LBSIM_FUSED_MT=$mt timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 \
      --workload $w >> $O/bench.jsonl 2>> $O/bench_err.log || exit 12
  done
done
cd /tmp && export TMPDIR=/tmp
for w in qmix sac-gru; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o $w --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 --workload $w > $O/prof_$w.log 2>&1 || exit 13
done
