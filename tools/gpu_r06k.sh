#!/bin/bash
# Round-6 diagnostics: policy kernels with the weight stream held in L1 (LBSIM_EXP_L1W timing
# variant, wrong results) against the shipped build, the eager / graph step comparison on one GPU
# state (tools/graph_gap_exp.py), and the single-env breakdown.   usage: bash tools/gpu_r06k.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06k}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/gpu_lib_ab.sh $TAG/sac cur l1w -- --workload sac-gru || exit 10
bash tools/gpu_lib_ab.sh $TAG/qmix cur l1w -- --workload qmix || exit 11
timeout -k 10 300 python tools/graph_gap_exp.py --rounds 2 > $O/graph_gap.jsonl 2> $O/graph_gap.err || exit 12
timeout -k 10 300 python tools/single_env_breakdown.py --steps 2000 > $O/single_env_breakdown.json 2> $O/breakdown.err || exit 13
