#!/bin/bash
# GPU box: SQ counters of the Monte-Carlo kernels (tools/sim_time.py --producer fused runs the
# producer, the decode+count kernel and the whole-iteration kernel).  usage: bash tools/sq_sim.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d /tmp/sqsim_${TAG} -o run -- python3 $R/tools/sim_time.py --producer fused > $R/gpurun_out/sqsim_${TAG}.log 2>&1 || exit 1
python3 $R/tools/sq_summary.py /tmp/sqsim_${TAG}/run_counter_collection.csv | grep -E "pl_sc_static|awgn_llr" > $R/gpurun_out/sqsim_$TAG.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU --output-format csv -d /tmp/grsim_${TAG} -o run -- python3 $R/tools/sim_time.py --producer fused > $R/gpurun_out/grsim_${TAG}.log 2>&1 || exit 1
python3 $R/tools/sq_summary.py /tmp/grsim_${TAG}/run_counter_collection.csv | grep -E "pl_sc_static|awgn_llr" >> $R/gpurun_out/sqsim_$TAG.txt
cat $R/gpurun_out/sqsim_$TAG.txt
