#!/bin/bash
# GPU box: SQ counters of the SCL subtree kernel (tools/scl_ab.py).  usage: bash tools/sq_scl.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/sq_$TAG -o run -- python3 $R/tools/scl_ab.py --kernels subtree --reps 1 "$@" > $R/gpurun_out/sq_$TAG.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_FP64 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/sq2_$TAG -o run -- python3 $R/tools/scl_ab.py --kernels subtree --reps 1 "$@" > $R/gpurun_out/sq2_$TAG.log 2>&1 || exit 1
python3 $R/tools/sq_summary.py $R/gpurun_out/sq_$TAG $R/gpurun_out/sq2_$TAG
