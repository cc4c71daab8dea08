#!/bin/bash
# Round-3 GPU pass: parity tests, smoke, bench (fused step = default, and the two-launch split for
# A/B), rocprofv3 kernel trace of the default bench.  usage: bash tools/gpu_r03.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r03}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 10; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 300 python bench.py "$@" > $O/bench.log 2>&1 || exit 12
for k in split fused split fused; do
  LBSIM_STEP_KERNEL=$k timeout -k 10 120 python bench.py --no-cpu-baseline "$@" >> $O/ab_$k.jsonl 2>> $O/ab.err || exit 13
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 "$@" > $O/prof_bench.log 2>&1 || exit 14
