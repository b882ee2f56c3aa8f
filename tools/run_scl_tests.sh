set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_mysn_gpu.py tests/test_scl_gpu.py -q -rf > gpurun_out/pytest_scl.log 2>&1
echo rc=$?
