#!/bin/bash
# PMC passes (each counter group its own rocprofv3 run; never combined with trace domains).
# usage: bash tools/gpu_pmc.sh <tag> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-pmc}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/pmc_list.txt 2>&1
B="$R/bench.py --no-cpu-baseline --steps 6 --warmup 2 $@"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/calf -o run --output-format csv -- python3 $R/tools/pmc_calib.py > $O/calf.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/calw -o run --output-format csv -- python3 $R/tools/pmc_calib.py > $O/calw.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/sq1 -o run --output-format csv -- python3 $B > $O/sq1.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $B > $O/sq2.log 2>&1
