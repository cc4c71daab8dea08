#!/bin/bash
# Round-6: the SAC actor at 16- vs 32-env tiles (LBSIM_FUSED_MT) now that its staging is one round
# trip, shipped build and phases build.   usage: bash tools/gpu_r06q.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06q}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/gpu_lib_ab.sh $TAG/sac cur:LBSIM_FUSED_MT=1 cur:LBSIM_FUSED_MT=2 -- --workload sac-gru || exit 10
bash tools/gpu_lib_ab.sh $TAG/qmix cur:LBSIM_FUSED_MT=1 -- --workload qmix || exit 11
for mt in 1 2; do
  echo "== MT $mt" >> $O/sac_phases.jsonl
  LBSIM_FUSED_MT=$mt LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_phases.so timeout -k 10 300 python tools/policy_phases.py --workload sac-gru >> $O/sac_phases.jsonl 2>> $O/phases.err || exit 12
done
