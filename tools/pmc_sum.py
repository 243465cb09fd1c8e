"""Sum rocprofv3 --pmc counter CSVs per kernel (all launches) and print one line per kernel."""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0]
        tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda kv: -max(kv[1].values())):
    if any(v > 0 for v in c.values()):
        line = " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items()))
        extra = ""
        if c.get("SQ_LDS_IDX_ACTIVE"):
            extra = f" conflict_frac={c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.3f}"
        print(f"{k[:60]:60s} {line}{extra}")
