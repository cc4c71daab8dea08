#!/bin/bash
# SQ counter passes of one bench shape (each group its own rocprofv3 run, no trace domains):
# issue / wait / instruction mix of the dynamics kernels.  usage: bash tools/gpu_pmc_wave.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-pmcw}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-graph --steps 6 --warmup 2 $@"
P="timeout -s KILL 240 rocprofv3"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/sq1 -o run --output-format csv -- python3 $B > $O/sq1.log 2>&1 &&
$P --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $B > $O/sq2.log 2>&1 &&
$P --pmc SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_LDS -d $O/sq3 -o run --output-format csv -- python3 $B > $O/sq3.log 2>&1
