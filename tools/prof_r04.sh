#!/bin/bash
# Round-4 profile evidence on the GPU box.  usage: bash tools/prof_r04.sh TAG
#  1. the driver's bench command (python bench.py) under rocprofv3 --kernel-trace --stats: kernel
#     statistics, the headline's timed window (tools/trace_window.py) and the durations of the
#     configs[1] / configs[3] launches and the single-wave probe (tools/trace_configs.py);
#  2. --pmc passes, each its own run: FETCH_SIZE, WRITE_SIZE (HBM traffic of the SC kernel);
#  3. SQ passes per decoder (VALU class counts, VALU thread-cycles, waits) for the VALU roofline
#     (tools/valu_roofline.py), and the same counters on the calibration kernels (valu_cycles).
# Every step runs under its own timeout; the first failure ends the script.
set -eo pipefail
TAG=${1:?usage: prof_r04.sh TAG}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
T=/tmp/${TAG}_prof
B="--no-cpu-baseline --no-sim-iteration --no-configs --settle-ms 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $T/bench -o bench -- python3 $R/bench.py > $O/${TAG}_bench_traced.json 2> $O/${TAG}_bench_traced.err
KT=$(find $T/bench -name "*kernel_trace.csv" | head -1)
cp $(find $T/bench -name "*kernel_stats.csv" | head -1) $O/${TAG}_bench_kernel_stats.csv
python3 $R/tools/trace_window.py $KT $O/${TAG}_bench_traced.json > $O/${TAG}_sc_trace_window.json
python3 $R/tools/trace_configs.py $KT > $O/${TAG}_trace_configs.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $T/pmc_$c -o run -- python3 $R/bench.py --steps 3 --warmup 1 $B > /dev/null 2> $O/${TAG}_pmc_$c.err
  cp $(find $T/pmc_$c -name "*counter_collection.csv") $O/${TAG}_pmc_sc_$c.csv
done
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
PB="SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
PC="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM"
for dec in sc scl; do
  for p in A B C; do
    eval "CS=\$P$p"
    timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d $T/sq_${dec}_$p -o run -- python3 $R/bench.py --decoder $dec --steps 5 --warmup 1 $B > /dev/null 2> $O/${TAG}_sq_${dec}_$p.err
    cp $(find $T/sq_${dec}_$p -name "*counter_collection.csv") $O/${TAG}_sq_${dec}_$p.csv
  done
done
for p in A B; do
  eval "CS=\$P$p"
  timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d $T/cal_$p -o run -- $R/tools/micro/valu_cycles > $O/${TAG}_valu_cycles_$p.txt 2> $O/${TAG}_valu_cycles_$p.err
  cp $(find $T/cal_$p -name "*counter_collection.csv") $O/${TAG}_valu_cycles_$p.csv
done
ls -la $O | grep $TAG
