"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (sum over
dispatches, dispatch count) into a small JSON -- run on the GPU box so the raw
CSV (one row per dispatch and counter) need not travel back."""
import csv
import glob
import json
import sys
from collections import defaultdict

src, dst = sys.argv[1], sys.argv[2]
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(src + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "").split("(")[0].replace("yrwi::", "")[:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
out = {k: {"dispatches": len(disp[k]), **{c: v for c, v in agg[k].items()}} for k in agg}
json.dump(out, open(dst, "w"), indent=1)
