# Same-process A/B timing of the SCL variant libraries (tools/scl_variants.py), no parity tests
# (variants may be timing diagnostics); configurations "FMODE FLAGS" as arguments.
cd $GRAFT_REPO_ROOT
for cfg in "$@"; do
  set -- $cfg
  echo "SCL_FMODE=$1 SCL_FLAGS=$2"
  SCL_FMODE=$1 SCL_FLAGS=$2 SCL_ROUNDS=${SCL_ROUNDS:-2} timeout -k 10 300 python -u tools/scl_variants.py time || exit $?
done
