#!/bin/bash
# round-1 first GPU pass: parity tests, smoke, bench, kernel-trace stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd $R
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
# 0 = pass, 1 = test failures (numerics); anything else (fault/abort/timeout) ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 10; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit 12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 > $R/gpurun_out/prof_bench.log 2>&1 || exit 13
