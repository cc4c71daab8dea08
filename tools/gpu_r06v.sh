#!/bin/bash
# Round-6 final pass of the committed tree: every GPU test and smoke(), the driver's bench command,
# then the single-env latency with its kernel trace (tools/gpu_latency_prof.sh).
#   usage: bash tools/gpu_r06v.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06v}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err || exit 12
bash tools/gpu_latency_prof.sh $TAG/latency || exit 13
