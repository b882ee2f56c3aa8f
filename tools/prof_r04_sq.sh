#!/bin/bash
# SQ counter passes only (tools/prof_r04.sh steps 3): the bench kernels of DECODERS (default
# "sc scl") and the calibration kernels.  usage: bash tools/prof_r04_sq.sh TAG [DECODERS]
set -eo pipefail
TAG=${1:?usage: prof_r04_sq.sh TAG [DECODERS]}
DECS=${2:-"sc scl"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
T=/tmp/${TAG}_prof
B="--no-cpu-baseline --no-sim-iteration --no-configs --settle-ms 0"
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
PB="SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
PC="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM"
for dec in $DECS; do
  for p in A B C; do
    eval "CS=\$P$p"
    timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d $T/sq_${dec}_$p -o run -- python3 $R/bench.py --decoder $dec --steps 5 --warmup 1 $B > /dev/null 2> $O/${TAG}_sq_${dec}_$p.err
    cp $(find $T/sq_${dec}_$p -name "*counter_collection.csv") $O/${TAG}_sq_${dec}_$p.csv
  done
done
for p in A B; do
  eval "CS=\$P$p"
  timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d $T/cal_$p -o run -- $R/tools/micro/valu_cycles > $O/${TAG}_valu_cycles_$p.txt 2> $O/${TAG}_valu_cycles_$p.err
  cp $(find $T/cal_$p -name "*counter_collection.csv") $O/${TAG}_valu_cycles_$p.csv
done
ls $O | grep $TAG
