#!/bin/bash
# GPU box: SQ_INSTS_VALU / SALU / wave cycles of each named SC variant (tools/sc_ab.py specs), one
# rocprofv3 pass per variant.  usage: bash tools/sq_variants_sc.sh TAG NAME...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d /tmp/sqv_${TAG}_$v -o run -- python3 $R/tools/sc_ab.py run $v --only --rounds 1 > $R/gpurun_out/sqv_${TAG}_$v.log 2>&1 || exit 1
  echo "== $v" >> $R/gpurun_out/sqv_$TAG.txt
  python3 $R/tools/sq_summary.py /tmp/sqv_${TAG}_$v/run_counter_collection.csv | grep pl_sc_static_f32 >> $R/gpurun_out/sqv_$TAG.txt
done
cat $R/gpurun_out/sqv_$TAG.txt
