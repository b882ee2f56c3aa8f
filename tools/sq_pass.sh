#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/avail.txt 2>&1 || true
for v in base d8; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d /tmp/sq_$v -o run -- python3 $R/tools/sc_ab.py run $v --only --rounds 1 > $R/gpurun_out/sq_$v.log 2>&1 || exit 1
  python3 $R/tools/sq_summary.py /tmp/sq_$v/run_counter_collection.csv | grep pl_sc_static_f32 >> $R/gpurun_out/sq_r02r.txt
done
