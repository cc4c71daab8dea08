#!/bin/bash
# Small-batch 8-lane groups: simulator parity (incl. the B = 8256 case and the wider-group child
# runs), smoke, then bench at 4096 x 4 / 8192 x 4 / 65536 x 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-s5j}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
: > $O/bench.jsonl
for a in "--batch 4096" "--batch 8192" "--batch 4096" "--batch 8192" ""; do
  timeout -k 10 120 python bench.py --no-cpu-baseline $a >> $O/bench.jsonl 2>> $O/bench.err || exit 12
done
