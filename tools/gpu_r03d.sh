#!/bin/bash
# Round-3 measurement pass: every BASELINE workload (policy glue after the step writes agent obs /
# state), the S = 8 trace replay, 4096 x 4, the single-env latency (both dynamics mappings) and
# rocprof kernel traces of the QMIX / SAC-GRU workloads.  usage: bash tools/gpu_r03d.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r03d}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/workloads.jsonl
for a in "--batch 4096" "--batch 4096 --dyn-mapping env" "--trace poisson_for_loop_rate_500 --servers 8" "--workload sac-gru" "--workload qmix" "--workload qmix --servers 64"; do
  echo "== $a" >> $O/workload_err.log
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $a >> $O/workloads.jsonl 2>> $O/workload_err.log || exit 21
done
timeout -k 10 300 python tools/single_env_latency.py --steps 2000 > $O/latency.jsonl 2>> $O/workload_err.log || exit 22
timeout -k 10 300 python tools/single_env_latency.py --steps 2000 --dyn-mapping env >> $O/latency.jsonl 2>> $O/workload_err.log || exit 23
cd /tmp && export TMPDIR=/tmp
for w in qmix sac-gru; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o $w --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 --workload $w > $O/prof_$w.log 2>&1 || exit 24
done
