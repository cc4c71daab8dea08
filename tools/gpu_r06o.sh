#!/bin/bash
# Round-6: dynamics prologues in two HBM round trips and the carried-in loop without flat loads --
# every GPU test, the headline A/B against the committed dynamics (base), the policy phase
# timelines, the single-env latency.   usage: bash tools/gpu_r06o.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06o}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
bash tools/gpu_lib_ab.sh $TAG/ab base cur -- || exit 11
for w in qmix sac-gru; do
  LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_phases.so timeout -k 10 300 python tools/policy_phases.py --workload $w >> $O/phases.jsonl 2>> $O/phases.err || exit 12
done
timeout -k 10 300 python tools/single_env_latency.py --steps 2000 > $O/latency.jsonl 2> $O/lat.err || exit 13
