#!/bin/bash
# One rocprofv3 --pmc pass (own run, kernel trace only) over a short isolated bench;
# per-kernel counter sums into gpurun_out/pmc/<tag>.csv (kernel, counter, total, dispatches, per dispatch).
#   bash tools/pmc_pass.sh <tag> "<COUNTER ...>" [bench args]
set -e
TAG=$1; CTRS=$2; shift 2
ARGS=${@:---steps 3 --warmup 1 --no-cpu --latency 0 --inflight 1 --legs none}
R=$(pwd)
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-include-regex "${PMC_KERNELS:-k_reduce|k_score|k_compact|k_probe}" --output-format csv -d /tmp/pmc_$TAG -o run -- python3 $R/bench.py $ARGS > /tmp/pmc_$TAG.log 2>&1
python3 - "$R/gpurun_out/pmc/$TAG.csv" /tmp/pmc_$TAG <<'PY'
import csv, glob, sys
from collections import defaultdict
tot = defaultdict(float); disp = defaultdict(set)
for f in glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
with open(sys.argv[1], "w") as o:
    o.write("kernel,counter,total,dispatches,per_dispatch\n")
    for (k, c), v in sorted(tot.items()):
        n = len(disp[k]) or 1
        o.write(f"\"{k}\",{c},{v:.0f},{n},{v / n:.1f}\n")
PY
