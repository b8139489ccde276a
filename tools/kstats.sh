#!/bin/bash
# Per-kernel average durations of one short isolated bench (rocprofv3 --kernel-trace --stats),
# summarised on the box into gpurun_out/<tag>_kstats.txt (raw traces stay in /tmp).
set -e
TAG=${1:-k}
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/kst
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --latency 0 --inflight 1 --legs none $KARGS > /tmp/kst.log 2>&1
python3 - "$R/gpurun_out/${TAG}_kstats.txt" <<'PY'
import csv, glob, sys
f = glob.glob("/tmp/kst/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
with open(sys.argv[1], "w") as o:
    for r in rows:
        o.write("%-50s %6s %10.1f us\n" % (r["Name"].split("(")[0][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
if [ -n "$KTRACE" ]; then  # per-dispatch durations of the kernels whose name contains $KTRACE
python3 - "$R/gpurun_out/${TAG}_ktrace.txt" "$KTRACE" <<'PY'
import csv, glob, sys
f = glob.glob("/tmp/kst/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if sys.argv[2] in r["Kernel_Name"]]
with open(sys.argv[1], "w") as o:
    for r in rows:
        o.write("%s %d %.1f\n" % (r["Kernel_Name"].split("(")[0], int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0),
                                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
fi
