#!/bin/bash
# GPU box: SQ counters of the bench's kernels.  usage: bash tools/sq_bench.sh TAG [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/sq_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/sq_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/sq2_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/sq2_$TAG.log 2>&1 || exit 1
echo sq_done
