#!/bin/bash
# The grid-size-selected 5-wave dynamics kernel: the simulator parity tests (incl. the > 4 waves per
# SIMD grids), then bench at 65536 x 4 (4-wave form), 65536 x 8 trace, 262144 x 4 (5-wave form).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-dyn5}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 10
: > $O/bench.jsonl
for a in "--batch 65536" "--trace poisson_for_loop_rate_500 --servers 8" "--batch 262144" "--workload sac-gru"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 $a >> $O/bench.jsonl 2>> $O/err.log || exit 11
done
