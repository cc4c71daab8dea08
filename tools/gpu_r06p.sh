#!/bin/bash
# Round-6: dynamics prologue with only the queued window entries loaded (in parallel) -- every GPU
# test, the headline A/B against the committed dynamics (base); the SAC actor with its staging
# reads removed (timing-only build, LBSIM_EXP_NOSTAGE) against the phases build.
#   usage: bash tools/gpu_r06p.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06p}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
bash tools/gpu_lib_ab.sh $TAG/ab base cur -- || exit 11
for v in phases nostage; do
  echo "== $v" >> $O/sac_phases.jsonl
  LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_$v.so timeout -k 10 300 python tools/policy_phases.py --workload sac-gru >> $O/sac_phases.jsonl 2>> $O/phases.err || exit 12
done
bash tools/gpu_lib_ab.sh $TAG/sac phases nostage -- --workload sac-gru || exit 13
