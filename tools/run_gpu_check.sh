set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.log 2>&1 && \
bash tools/gpu_profile.sh r01c
