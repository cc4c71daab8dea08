#!/bin/bash
# Round-6 evidence pass: rocprofv3 kernel trace (--stats) of the default bench and of the driver's
# command, then the PMC passes of tools/gpu_pmc.sh (FETCH / WRITE with their calibration, SQ and
# VALU-class counters; each group its own run, never with trace domains).  The VALU issue prices
# come from the committed micro-benchmark (profiles/r03/ubench_valu.jsonl).
#   usage: bash tools/gpu_r06_prof.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06prof}
O=$R/gpurun_out/$TAG
mkdir -p $O
cp $R/profiles/r03/ubench_valu.jsonl $O/
cd /tmp && export TMPDIR=/tmp
P="timeout -s KILL 240 rocprofv3"
$P --kernel-trace --stats -d $O/trace_default -o run --output-format csv -- python3 $R/bench.py --no-graph --no-cpu-baseline > $O/trace_default.json 2> $O/trace_default.err || exit 20
$P --kernel-trace --stats -d $O/trace_driver -o run --output-format csv -- python3 $R/bench.py --no-graph --no-cpu-baseline --steps 20 --warmup 5 > $O/trace_driver.json 2> $O/trace_driver.err || exit 21
B="$R/bench.py --no-cpu-baseline --no-graph --steps 20 --warmup 5"
$P --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/calf -o run --output-format csv -- python3 $R/tools/pmc_calib.py > $O/calf.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/calw -o run --output-format csv -- python3 $R/tools/pmc_calib.py > $O/calw.log 2>&1 &&
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/sq1 -o run --output-format csv -- python3 $B > $O/sq1.log 2>&1 &&
$P --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $B > $O/sq2.log 2>&1 &&
$P --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU -d $O/vc1 -o run --output-format csv -- python3 $B > $O/vc1.log 2>&1 &&
$P --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE -d $O/vc2 -o run --output-format csv -- python3 $B > $O/vc2.log 2>&1
