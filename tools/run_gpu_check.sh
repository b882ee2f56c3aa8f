#!/bin/bash
# GPU box: full GPU test suite, smoke, bench (N=1) and the rocprofv3 profile of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.log 2>&1 && \
bash tools/gpu_profile.sh ${PROF_TAG:-r01d}
