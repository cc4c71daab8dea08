#!/bin/bash
# Round-6: phase timelines of the policy kernels (LBSIM_EXP_PHASES build) and the driver's bench
# command with 20 steps per captured graph.   usage: bash tools/gpu_r06m.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06m}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for w in qmix sac-gru; do
  LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_phases.so timeout -k 10 300 python tools/policy_phases.py --workload $w >> $O/phases.jsonl 2>> $O/phases.err || exit 10
done
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err || exit 11
