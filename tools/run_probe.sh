#!/bin/bash
# GPU box: static_probe timing (+ SQ counters of the named variant when PROBE_SQ is set).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
K=$1; N=$2; shift 2
timeout -k 10 300 python tools/static_probe.py run $K $N "$@" > gpurun_out/probe.log 2>&1 || exit 1
if [ -n "$PROBE_SQ" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/sq_probe -o run -- python3 $R/tools/static_probe.py run $K $N $PROBE_SQ > $R/gpurun_out/sq_probe.log 2>&1 || exit 1
fi
echo probe_done
