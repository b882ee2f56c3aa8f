#!/bin/bash
# SCL bench kernel evidence after its round-4 changes: kernel trace + stats of `bench.py --decoder
# scl`, and the FETCH_SIZE / WRITE_SIZE passes (each its own run) for profiles/traffic.json
# (tools/pmc_summary.py TAG scl).  usage: bash tools/prof_r04_scl.sh TAG
set -eo pipefail
TAG=${1:?usage: prof_r04_scl.sh TAG}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
T=/tmp/${TAG}_prof
B="--no-cpu-baseline --no-sim-iteration --no-configs --settle-ms 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/scl -o scl -- python3 $R/bench.py --decoder scl --no-cpu-baseline > $O/${TAG}_bench_scl_traced.json 2> $O/${TAG}_bench_scl_traced.err
cp $(find $T/scl -name "*kernel_stats.csv" | head -1) $O/${TAG}_scl_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $T/pmc_$c -o run -- python3 $R/bench.py --decoder scl --steps 3 --warmup 1 $B > /dev/null 2> $O/${TAG}_pmc_scl_$c.err
  cp $(find $T/pmc_$c -name "*counter_collection.csv") $O/${TAG}_pmc_scl_$c.csv
done
ls $O | grep $TAG
