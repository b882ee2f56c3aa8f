#!/bin/bash
# GPU box: SQ / GRBM counters of named SC A/B variants (tools/sc_ab.py specs), one rocprofv3 pass
# per variant and counter set.  usage: bash tools/sq_pass.sh TAG NAME...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d /tmp/sq_${TAG}_$v -o run -- python3 $R/tools/sc_ab.py run $v --only --rounds 1 > $R/gpurun_out/sq_${TAG}_$v.log 2>&1 || exit 1
  python3 $R/tools/sq_summary.py /tmp/sq_${TAG}_$v/run_counter_collection.csv | grep pl_sc_static_f32 >> $R/gpurun_out/sq_$TAG.txt
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU --output-format csv -d /tmp/gr_${TAG}_$v -o run -- python3 $R/tools/sc_ab.py run $v --only --rounds 1 > $R/gpurun_out/gr_${TAG}_$v.log 2>&1 || exit 1
  python3 $R/tools/sq_summary.py /tmp/gr_${TAG}_$v/run_counter_collection.csv | grep pl_sc_static_f32 >> $R/gpurun_out/sq_$TAG.txt
  python3 - /tmp/gr_${TAG}_$v >> $R/gpurun_out/sq_$TAG.txt <<'PY'
import csv, glob, sys
d = sys.argv[1]
kt = [r for f in glob.glob(d + "/*kernel_trace.csv") for r in csv.DictReader(open(f)) if "pl_sc_static_f32" in r["Kernel_Name"]]
cc = [r for f in glob.glob(d + "/*counter_collection.csv") for r in csv.DictReader(open(f)) if "pl_sc_static_f32" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
if kt and cc:
    ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt) / len(kt)
    cyc = sum(float(r["Counter_Value"]) for r in cc) / len(cc)
    print(f"  kernel {ns/1e3:.2f} us (trace avg, {len(kt)} launches), GRBM_GUI_ACTIVE {cyc:.0f} cycles -> {cyc/ns:.3f} GHz")
PY
done
cat $R/gpurun_out/sq_$TAG.txt
