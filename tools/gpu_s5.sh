#!/bin/bash
# Round-2 session-5 GPU pass: tests + smoke + bench + kernel trace (gpu_check.sh), then the
# stream-split experiment (tools/stream_split_exp.py) at 65536 x 4 and 65536 x 8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r02s5}
O=$R/gpurun_out/$TAG
bash $R/tools/gpu_check.sh $TAG || exit $?
cd $R
timeout -k 10 240 python tools/stream_split_exp.py --parts 1,2,4,1 > $O/stream_split_s4.jsonl 2> $O/stream_split.err || exit 30
timeout -k 10 240 python tools/stream_split_exp.py --servers 8 --parts 1,2,1 > $O/stream_split_s8.jsonl 2>> $O/stream_split.err || exit 31
