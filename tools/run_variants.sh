#!/bin/bash
# GPU box: time every built SC variant in one process, then SQ counters for the named ones.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 300 python tools/variants.py time --rounds 2 > gpurun_out/variants.log 2>&1 || exit 1
if [ $# -gt 0 ]; then bash tools/sq_variants.sh "$@" || exit 1; fi
echo variants_done
