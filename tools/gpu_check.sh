#!/bin/bash
# GPU pass: parity tests (must be green), smoke, bench, rocprofv3 kernel-trace/stats.
# usage: bash tools/gpu_check.sh <tag> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-run}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 10; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py "$@" > $O/bench.log 2>&1 || exit 12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 "$@" > $O/prof_bench.log 2>&1 || exit 13
