"""Summarise rocprofv3 SQ counter CSVs per kernel (per-wave averages)."""
import csv, collections, glob, sys
for f in sys.argv[1:]:
    for path in glob.glob(f if f.endswith(".csv") else f + "/*counter_collection.csv"):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        cnt = collections.defaultdict(lambda: collections.Counter())
        for r in csv.DictReader(open(path)):
            kn = r["Kernel_Name"][:60]
            agg[kn][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[kn][r["Counter_Name"]] += 1
        for kn, d in agg.items():
            d = {c: v / cnt[kn][c] for c, v in d.items()}
            w = d.get("SQ_WAVES", 0)
            if not w:
                continue
            print(path.split("/")[-2], kn, {c: round(v / w, 1) for c, v in sorted(d.items()) if c != "SQ_WAVES"}, "waves", w)
