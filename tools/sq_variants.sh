#!/bin/bash
# SQ counters per SC variant (GPU box).  usage: bash tools/sq_variants.sh name1 name2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/sqv_$v -o run -- python3 $R/tools/variants.py time --only $v --reps 2 --rounds 1 > $R/gpurun_out/sqv_$v.log 2>&1 || exit 1
done
echo done
