#!/bin/bash
# Round-end GPU pass (one gpurun call, every step under its own time limit, chained):
#   1. pytest -m gpu (all parity tests) and smoke()
#   2. the default bench line (bench.py, N = 1: headline, graph leg, CPU baseline points)
#   3. a rocprofv3 kernel trace of the headline bench
#   4. one bench line per BASELINE workload (+ graph legs): 4096 x 4, 4096 x 8, configs[2] trace 65536 x 8,
#      configs[3] SAC-GRU, configs[4] QMIX (4 x 4 and 4 x 16)
#   5. async env groups + late-episode legs, the single-env latency, the 4k-512k batch sweep
# usage: bash tools/gpu_round.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-round}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 10 > $O/prof_bench.log 2>&1 || exit 13
cd $R
: > $O/workloads.jsonl
for a in "--batch 4096" "--batch 4096 --servers 8" "--trace poisson_for_loop_rate_500 --servers 8" "--workload sac-gru" "--workload qmix" "--workload qmix --servers 64"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $a >> $O/workloads.jsonl 2>> $O/workloads.err || exit 14
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --async-groups 2 --late-episode 1000,5000 > $O/async_late.json 2>> $O/workloads.err || exit 15
timeout -k 10 300 python tools/single_env_latency.py --steps 2000 > $O/single_env_latency.json 2>> $O/workloads.err || exit 16
timeout -k 10 300 python tools/single_env_breakdown.py --steps 2000 > $O/single_env_breakdown.json 2>> $O/workloads.err || exit 18
bash tools/gpu_sweep.sh $TAG --no-graph || exit 17
