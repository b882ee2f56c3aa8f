# Instruction-cache counters of the SCL and SC bench kernels (development aid).  usage: bash tools/icache_pass.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="--no-cpu-baseline --no-sim-iteration --no-configs --settle-ms 0 --steps 3 --warmup 1"
for dec in scl sc; do
  timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d /tmp/ic_${dec} -o run -- python3 $R/bench.py --decoder $dec $B > /dev/null 2> $O/${TAG}_ic_${dec}.err || exit 1
  cp $(find /tmp/ic_${dec} -name "*counter_collection.csv") $O/${TAG}_ic_${dec}.csv
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d /tmp/if_${dec} -o run -- python3 $R/bench.py --decoder $dec $B > /dev/null 2> $O/${TAG}_if_${dec}.err || exit 1
  cp $(find /tmp/if_${dec} -name "*counter_collection.csv") $O/${TAG}_if_${dec}.csv
done
python3 - $O $TAG <<'PY'
import csv, sys, collections
O, TAG = sys.argv[1], sys.argv[2]
for dec, kern in (("scl", "scl_tree_kernel<8, 4, 0, false>"), ("sc", "pl_sc_static_f32")):
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in (f"{O}/{TAG}_ic_{dec}.csv", f"{O}/{TAG}_if_{dec}.csv"):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for d in per.values():
            for c, v in d.items():
                tot[c] += v / len(per)
    print(dec, {c: round(v) for c, v in sorted(tot.items())})
PY
