# Same-process A/B of the SCL variant libraries (tools/scl_variants.py) for min-sum, exact f and
# exact f + fast-SCL (the my_sn default), no parity tests (variants are timing probes).
cd $GRAFT_REPO_ROOT
for cfg in "0 0" "1 0" "1 4"; do
  set -- $cfg
  echo "SCL_FMODE=$1 SCL_FLAGS=$2"
  SCL_FMODE=$1 SCL_FLAGS=$2 SCL_ROUNDS=2 timeout -k 10 300 python -u tools/scl_variants.py time || exit $?
done
