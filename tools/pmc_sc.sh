#!/bin/bash
# GPU box: one rocprofv3 PMC pass over the SC bench (counters given as arguments), summary per
# kernel into gpurun_out/pmc_<TAG>.txt.  usage: bash tools/pmc_sc.sh TAG COUNTER...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $R/gpurun_out/pmc_$TAG.log 2>&1 || exit 1
python3 $R/tools/sq_summary.py /tmp/pmc_$TAG/*/run_counter_collection.csv /tmp/pmc_$TAG/run_counter_collection.csv 2>/dev/null | grep -E "pl_sc_static|scl_tree" > $R/gpurun_out/pmc_$TAG.txt
cat $R/gpurun_out/pmc_$TAG.txt
