#!/bin/bash
# Final pass of a committed tree: every GPU test, smoke(), the driver's bench command, the default
# bench line and a rocprofv3 kernel trace (+ stats) of the default bench command.
# usage: bash tools/gpu_final.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-final}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit 12
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 13
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-graph > $O/prof_bench.log 2>&1 || exit 14
