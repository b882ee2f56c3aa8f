#!/bin/bash
# Profile evidence of the bench kernels on the GPU box.  usage: bash tools/prof_pass.sh TAG
#  1. the driver's bench command (python bench.py) under rocprofv3 --kernel-trace --stats: kernel
#     statistics, the headline's timed window (tools/trace_window.py) and the durations of the
#     configs[1] / configs[3] / mysn_sc_exact / mysn_scl launches (tools/trace_configs.py);
#  2. --pmc passes, each its own run: FETCH_SIZE and WRITE_SIZE of the SC headline kernel, of the
#     SCL bench kernel (its private-memory VCache traffic) and of my_sn SCL_Dec's default kernel;
#  3. SQ passes (VALU class counts, waits) of the exact-f SC kernel (my_sn SC_Dec at (512,1024)),
#     the min-sum SC kernel, the SCL kernel and my_sn SCL_Dec's default (exact f + fast-SCL).
# SQ_ONLY=1 runs step 3 only, SQ_DECS="..." picks its decoders; CAL=1 adds the VALU issue-cost
# calibration (tools/micro/valu_cycles.hip, built here from its source).
# Every step runs under its own timeout; the first failure ends the script.
set -eo pipefail
TAG=${1:?usage: prof_pass.sh TAG}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
T=/tmp/${TAG}_prof
B="--no-cpu-baseline --no-sim-iteration --no-configs --settle-ms 0"
dec_args() {
  case $1 in
    scx) echo "--decoder sc --fmode 1" ;;
    sclx) echo "--decoder scl --fmode 1 --fast-scl" ;;
    *) echo "--decoder $1" ;;
  esac
}
if [ -z "$SQ_ONLY" ]; then
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $T/bench -o bench -- python3 $R/bench.py > $O/${TAG}_bench_traced.json 2> $O/${TAG}_bench_traced.err
KT=$(find $T/bench -name "*kernel_trace.csv" | head -1)
cp $(find $T/bench -name "*kernel_stats.csv" | head -1) $O/${TAG}_bench_kernel_stats.csv
python3 $R/tools/trace_window.py $KT $O/${TAG}_bench_traced.json > $O/${TAG}_sc_trace_window.json
python3 $R/tools/trace_configs.py $KT > $O/${TAG}_trace_configs.json
for dec in sc scl sclx; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $T/pmc_${dec}_$c -o run -- python3 $R/bench.py $(dec_args $dec) --steps 3 --warmup 1 $B > /dev/null 2> $O/${TAG}_pmc_${dec}_$c.err
    cp $(find $T/pmc_${dec}_$c -name "*counter_collection.csv") $O/${TAG}_pmc_${dec}_$c.csv
  done
done
fi
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
PB="SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
PC="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM"
for dec in ${SQ_DECS:-scx sc scl sclx}; do
  for p in A B C; do
    eval "CS=\$P$p"
    KTF=""
    [ $p = B ] && KTF="--kernel-trace"  # pass B: GRBM_GUI_ACTIVE with the dispatch durations (the clock)
    timeout -s KILL 120 rocprofv3 $KTF --pmc $CS --output-format csv -d $T/sq_${dec}_$p -o run -- python3 $R/bench.py $(dec_args $dec) --steps 5 --warmup 1 $B > /dev/null 2> $O/${TAG}_sq_${dec}_$p.err
    cp $(find $T/sq_${dec}_$p -name "*counter_collection.csv") $O/${TAG}_sq_${dec}_$p.csv
    [ $p = B ] && cp $(find $T/sq_${dec}_$p -name "*kernel_trace.csv") $O/${TAG}_sq_${dec}_B_trace.csv
  done
done
if [ -n "$CAL" ]; then
  # the calibration kernels' clock: GRBM_GUI_ACTIVE cycles per dispatch against its trace duration
  timeout -k 10 120 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 $R/tools/micro/valu_cycles.hip -o /tmp/valu_cycles
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $T/cal -o run -- /tmp/valu_cycles > $O/${TAG}_valu_cycles.txt 2> $O/${TAG}_valu_cycles.err
  cp $(find $T/cal -name "*counter_collection.csv") $O/${TAG}_valu_cycles_pmc.csv
  cp $(find $T/cal -name "*kernel_trace.csv") $O/${TAG}_valu_cycles_trace.csv
fi
ls -la $O | grep $TAG
