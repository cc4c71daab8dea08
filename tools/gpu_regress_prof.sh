#!/bin/bash
# Kernel traces of the round-2 tree (expl/r02) and this tree, same box, headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-regprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r02 -o r02 --output-format csv -- python3 $R/expl/r02/bench.py --no-cpu-baseline --steps 50 --warmup 10 > $O/r02.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03 -o r03 --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 10 > $O/r03.log 2>&1 || exit 15
