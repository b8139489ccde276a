#!/bin/bash
# gather microbenchmark: timing, then one PMC pass of L2->HBM read request sizes
set -e
R=$(pwd)
mkdir -p $R/gpurun_out/micro
timeout -k 10 60 $R/tools/micro/gather > $R/gpurun_out/micro/gather_time.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d /tmp/pmc_g -o run -- $R/tools/micro/gather > /tmp/pmc_g.log 2>&1
python3 - $R/gpurun_out/micro/gather_pmc.txt /tmp/pmc_g <<'PY'
import csv, glob, sys
from collections import defaultdict
tot = defaultdict(float); cnt = defaultdict(set)
for f in glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        cnt[k].add(r.get("Dispatch_Id"))
with open(sys.argv[1], "w") as o:
    for (k, c), v in sorted(tot.items()):
        o.write(f"{k:40s} {c:28s} {v / max(1, len(cnt[k])):14.0f} per launch\n")
PY
