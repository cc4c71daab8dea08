#!/bin/bash
# PMC passes of the default bench (each counter group its own rocprofv3 run, never combined with
# trace domains) + the VALU issue micro-benchmark.  usage: bash tools/gpu_pmc.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-pmc}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 ./tools/ubench_valu > $O/ubench_valu.jsonl 2> $O/ubench_valu.err || exit 9
cd /tmp && export TMPDIR=/tmp
# the driver's bench command (--steps 20 --warmup 5, pre-warm on) without the graph leg and the CPU
# baseline, which run after the timed region; tools/pmc_traffic.py / pmc_valu.py --steps 20
# --warmup 5 keep the timed launches (and their exact accounting replay) only
B="$R/bench.py --no-cpu-baseline --no-graph --steps 20 --warmup 5 $@"
P="timeout -s KILL 240 rocprofv3"
$P --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.log 2>&1 &&
$P --pmc FETCH_SIZE -d $O/calf -o run --output-format csv -- python3 $R/tools/pmc_calib.py > $O/calf.log 2>&1 &&
$P --pmc WRITE_SIZE -d $O/calw -o run --output-format csv -- python3 $R/tools/pmc_calib.py > $O/calw.log 2>&1 &&
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/sq1 -o run --output-format csv -- python3 $B > $O/sq1.log 2>&1 &&
$P --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- python3 $B > $O/sq2.log 2>&1 &&
$P --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU -d $O/vc1 -o run --output-format csv -- python3 $B > $O/vc1.log 2>&1 &&
$P --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE -d $O/vc2 -o run --output-format csv -- python3 $B > $O/vc2.log 2>&1
