#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of one isolated bench
# configuration: tools/kstats_cfg.sh <tag> <bench args...>  ->  gpurun_out/<tag>_kstats.txt
set -e
TAG=$1
shift
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_$TAG -o run -- python3 $R/bench.py --no-cpu --latency 0 --inflight 1 --legs none "$@" > $R/gpurun_out/${TAG}_kst.log 2>&1
python3 - "$R/gpurun_out/${TAG}_kstats.txt" /tmp/kst_$TAG <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
with open(sys.argv[1], "w") as o:
    for r in rows:
        o.write("%-50s %6s %10.1f us %10.1f ms total\n" % (r["Name"].split("(")[0][:50], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
