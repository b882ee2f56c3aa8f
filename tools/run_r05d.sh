# Round-5 GPU check d: the whole GPU suite (exact-f root mode, med3 clip), smoke, micros, bench.
# Every step under its own timeout; the first failure ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r05d}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread -p no:cacheprovider > $O/${T}_pytest_gpu.txt 2>&1 || { echo pytest failed; grep -E "FAILED|Error" $O/${T}_pytest_gpu.txt | head -20; tail -5 $O/${T}_pytest_gpu.txt; exit 1; }
tail -2 $O/${T}_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.txt 2>&1 || { cat $O/${T}_smoke.txt; exit 1; }
timeout -k 10 120 ./tools/micro/chain_latency > $O/${T}_chain_latency.txt 2>&1 || { cat $O/${T}_chain_latency.txt; exit 1; }
timeout -k 10 60 ./tools/micro/x2_check > $O/${T}_x2_check.txt 2>&1; cat $O/${T}_x2_check.txt
timeout -k 10 120 ./tools/micro/valu_cycles > $O/${T}_valu_cycles.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/${T}_bench_sc.json 2> $O/${T}_bench_sc.err || { tail -5 $O/${T}_bench_sc.err; exit 1; }
cat $O/${T}_chain_latency.txt
tail -c 2500 $O/${T}_bench_sc.json
