# SCL subtree kernel: parity tests, then same-process A/B timing against _variants/libscl_*.so
# at each PL_SCL_VIRTUAL setting given as arguments (default: 3 4).
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_scl_gpu.py tests/test_mysn_gpu.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_scl.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_scl.log
[ $rc -eq 0 ] || exit $rc
for v in ${@:-3 4}; do
  echo "PL_SCL_VIRTUAL=$v"
  PL_SCL_VIRTUAL=$v timeout -k 10 300 python -u tools/scl_variants.py time || exit $?
done
