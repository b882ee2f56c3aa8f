#!/bin/bash
# SQ VALU counter passes of both bench kernels (one rocprofv3 --pmc run each, as in
# tools/prof_r03.sh step 3), for tools/sq_roofline.py.  usage: bash tools/sq_r03.sh TAG
set -eo pipefail
TAG=${1:?usage: sq_r03.sh TAG}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
T=/tmp/${TAG}_sq
for dec in sc scl; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $T/sq_$dec -o run -- python3 $R/bench.py --decoder $dec --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-sim-iteration > /dev/null 2> $O/${TAG}_sq_$dec.err
  cp $(find $T/sq_$dec -name "*counter_collection.csv") $O/${TAG}_sq_$dec.csv
done
ls -la $O | grep $TAG
