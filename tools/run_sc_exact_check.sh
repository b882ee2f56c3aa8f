# exact-f SC: parity suites (statistical gates, oracle), then the timing of tools/quick_sc_time.py
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_exactf_gpu.py tests/test_sc_gpu.py tests/test_mysn_gpu.py tests/test_polar5g_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sc_exact.log 2>&1
rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/pytest_sc_exact.log
[ $rc -eq 0 ] || exit $rc
SC_FMODE=1 timeout -k 10 200 python tools/quick_sc_time.py
