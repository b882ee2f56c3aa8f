# exact-f SCL: parity tests of the release library, then same-process A/B timing of the variant
# libraries (tools/scl_variants.py) for exact f and exact f + fast-SCL (the my_sn default).
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_scl_gpu.py tests/test_mysn_gpu.py tests/test_exactf_gpu.py tests/test_polar5g_gpu.py tests/test_sim_sharded_gpu.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_scl_exact.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_scl_exact.log
[ $rc -eq 0 ] || exit $rc
for cfg in "1 0" "1 4" "0 0"; do
  set -- $cfg
  echo "SCL_FMODE=$1 SCL_FLAGS=$2"
  SCL_WS_AB=1 SCL_FMODE=$1 SCL_FLAGS=$2 SCL_ROUNDS=2 timeout -k 10 300 python -u tools/scl_variants.py time || exit $?
done
