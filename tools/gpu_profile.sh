#!/bin/bash
# Profile the bench on the GPU box: kernel trace + stats, then two PMC passes (FETCH_SIZE, WRITE_SIZE).
# usage: bash tools/gpu_profile.sh <tag> [bench args...]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 3 "$@" > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > $OUT/bench_write.log 2>&1
echo profile_done
