# Round-5 GPU check: the whole GPU suite, smoke, then timings of the exact-f decoders and the
# bench lines (SC default, SCL); every step under its own timeout, the first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?usage: run_r05_check.sh TAG}
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 120 --timeout-method thread -p no:cacheprovider > $O/${TAG}_pytest_gpu.txt 2>&1 || { echo pytest failed; tail -5 $O/${TAG}_pytest_gpu.txt; exit 1; }
tail -1 $O/${TAG}_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.txt 2>&1 || exit 1
timeout -k 10 200 python tools/mysn_time.py > $O/${TAG}_mysn_time.txt 2>&1 || exit 1
SC_FMODE=1 timeout -k 10 200 python tools/quick_sc_time.py > $O/${TAG}_sc_exact_time.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/${TAG}_bench_sc.json 2> $O/${TAG}_bench_sc.err || exit 1
timeout -k 10 300 python bench.py --decoder scl > $O/${TAG}_bench_scl.json 2> $O/${TAG}_bench_scl.err || exit 1
cat $O/${TAG}_mysn_time.txt $O/${TAG}_sc_exact_time.txt
