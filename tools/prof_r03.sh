#!/bin/bash
# Round-3 profile evidence on the GPU box.  usage: bash tools/prof_r03.sh TAG
#  1. the driver's bench command (python bench.py --gpus 1 --steps 20 --warmup 5) under
#     rocprofv3 --kernel-trace --stats: the kernel trace, its statistics, and the timed window
#     picked out of the trace (tools/trace_window.py) next to the bench line's HIP-event figure;
#  2. the SCL bench line and its kernel statistics;
#  3. rocprofv3 --pmc passes, each in its own run: FETCH_SIZE, WRITE_SIZE (SC), and one SQ pass per
#     decoder (SQ_INSTS_VALU ... GRBM_GUI_ACTIVE) for the VALU roofline (tools/valu_roofline.py).
# Every step runs under its own timeout; the first failure ends the script.
set -eo pipefail
TAG=${1:?usage: prof_r03.sh TAG}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
T=/tmp/${TAG}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/sc -o sc -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/${TAG}_bench_sc_traced.json 2> $O/${TAG}_bench_sc_traced.err
KT=$(find $T/sc -name "*kernel_trace.csv" | head -1)
cp $(find $T/sc -name "*kernel_stats.csv" | head -1) $O/${TAG}_sc_kernel_stats.csv
python3 $R/tools/trace_window.py $KT $O/${TAG}_bench_sc_traced.json > $O/${TAG}_sc_trace_window.json
python3 - "$KT" "$O/${TAG}_sc_trace_timed.csv" << 'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
kn = lambda raw: re.sub(r"^(void )?(\(anonymous namespace\)::)?", "", raw.strip()).split("(")[0]
keep = [r for r in rows if "pl_sc_static_f32" in r["Kernel_Name"] or "awgn_llr_kernel" in r["Kernel_Name"]]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "duration_ns"])
    for r in sorted(keep, key=lambda r: int(r["Start_Timestamp"])):
        w.writerow([kn(r["Kernel_Name"]), r["Start_Timestamp"], r["End_Timestamp"],
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"])])
PY
timeout -k 10 300 python3 $R/bench.py --decoder scl > $O/${TAG}_bench_scl.json 2> $O/${TAG}_bench_scl.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/scl -o scl -- python3 $R/bench.py --decoder scl --steps 10 --no-cpu-baseline > $O/${TAG}_prof_scl.json 2> $O/${TAG}_prof_scl.err
cp $(find $T/scl -name "*kernel_stats.csv" | head -1) $O/${TAG}_scl_kernel_stats.csv
for dec in sc scl; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $T/pmc_${dec}_$c -o run -- python3 $R/bench.py --decoder $dec --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-sim-iteration > /dev/null 2> $O/${TAG}_pmc_${dec}_$c.err
    cp $(find $T/pmc_${dec}_$c -name "*counter_collection.csv") $O/${TAG}_pmc_${dec}_$c.csv
  done
done
for dec in sc scl; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $T/sq_$dec -o run -- python3 $R/bench.py --decoder $dec --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-sim-iteration > /dev/null 2> $O/${TAG}_sq_$dec.err
  cp $(find $T/sq_$dec -name "*counter_collection.csv") $O/${TAG}_sq_$dec.csv
done
ls -la $O
