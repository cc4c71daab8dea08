#!/bin/bash
# Round-6: kernel trace of the eager / graph step comparison (tools/graph_gap_exp.py: per-kernel
# durations inside and outside the replayed graph), and the SAC actor at 8 waves per SIMD
# (LBSIM_SAC_WPE=8 build) against the shipped one.   usage: bash tools/gpu_r06l.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06l}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/gpu_lib_ab.sh $TAG/sac cur sacw8 -- --workload sac-gru || exit 10
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gg -o gg --output-format csv -- python3 $R/tools/graph_gap_exp.py --rounds 2 > $O/graph_gap.jsonl 2> $O/graph_gap.err || exit 11
