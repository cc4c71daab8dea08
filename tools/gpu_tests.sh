#!/bin/bash
# pytest -m gpu (every parity test) and smoke(), each under its own limit.
# usage: bash tools/gpu_tests.sh <tag> [pytest selection args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-tests}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
SEL=${@:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
