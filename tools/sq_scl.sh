#!/bin/bash
# GPU box: SQ counters of the SCL subtree kernel (tools/scl_ab.py).  usage: bash tools/sq_scl.sh TAG [scl_ab args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32" \
           "SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d /tmp/sq${i}_$TAG -o run -- python3 $R/tools/scl_ab.py --kernels subtree --reps 1 "$@" > $R/gpurun_out/sq${i}_$TAG.log 2>&1 || exit 1
done
python3 $R/tools/sq_summary.py /tmp/sq1_$TAG /tmp/sq2_$TAG /tmp/sq3_$TAG | tee $R/gpurun_out/sq_scl_$TAG.txt
