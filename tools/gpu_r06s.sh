#!/bin/bash
# Round-6 pass: every GPU test and smoke(), the driver's bench command and the default bench on
# the current tree (SAC at 32-env tiles), then the QMIX first-GRU-weights order A/B (qlate) with
# phase timelines.   usage: bash tools/gpu_r06s.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06s}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err || exit 12
timeout -k 10 600 python bench.py > $O/bench_default.json 2>> $O/bench.err || exit 13
bash tools/gpu_lib_ab.sh $TAG/qmix eps0 cur eps1q -- --workload qmix || exit 14
for v in phases qlatep; do
  echo "== $v" >> $O/qmix_phases.jsonl
  LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_$v.so timeout -k 10 300 python tools/policy_phases.py --workload qmix >> $O/qmix_phases.jsonl 2>> $O/phases.err || exit 15
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 10 --workload sac-gru > $O/sac.json 2>> $O/bench.err || exit 16
