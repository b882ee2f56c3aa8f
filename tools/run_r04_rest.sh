# Round-4 GPU check without the test suite: smoke, exact-f timings, the bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?usage: run_r04_rest.sh TAG}
O=gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.txt 2>&1 || exit 1
timeout -k 10 200 python tools/mysn_time.py > $O/${TAG}_mysn_time.txt 2>&1 || exit 1
SC_FMODE=1 timeout -k 10 200 python tools/quick_sc_time.py > $O/${TAG}_sc_exact_time.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/${TAG}_bench_sc.json 2> $O/${TAG}_bench_sc.err || exit 1
cat $O/${TAG}_smoke.txt $O/${TAG}_mysn_time.txt $O/${TAG}_sc_exact_time.txt $O/${TAG}_bench_sc.json
