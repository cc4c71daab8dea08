#!/bin/bash
# Round-6 closing pass: every GPU test and smoke() on the final tree, the driver's bench command and
# the SAC-GRU workload line.   usage: bash tools/gpu_r06x.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06x}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err || exit 12
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --workload sac-gru > $O/sac.json 2>> $O/bench.err || exit 13
