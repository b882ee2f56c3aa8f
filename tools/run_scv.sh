#!/bin/bash
# GPU box: tools/sc_variants.py run <names...>
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 400 python tools/sc_variants.py run "$@" > gpurun_out/scv.log 2>&1 || exit 1
echo scv_done
