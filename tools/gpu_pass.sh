#!/bin/bash
# One GPU call of a working tree, every step under its own limit, chained:
#   1. pytest -m gpu (all parity tests) and smoke()
#   2. the default bench line, then the driver's exact command
#   3. a rocprofv3 kernel-trace summary of the headline bench
#   4. (PMC=1) the FETCH/WRITE and SQ/VALU counter passes of tools/gpu_pmc.sh at 65536 x 4
# usage: [PMC=1] bash tools/gpu_pass.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-pass}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 12
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_cmd.json 2>> $O/bench.err || exit 13
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-graph --steps 30 > $O/prof_bench.log 2>&1 || exit 14
cd $R
if [ "${PMC:-0}" == "1" ]; then
  bash tools/gpu_pmc.sh $TAG/pmc || exit 15
fi
