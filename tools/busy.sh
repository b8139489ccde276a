#!/bin/bash
# GPU busy fraction of the default (two batches in flight) C2 bench: kernel trace of a
# bench run, then over the query kernels of the last half of the run: union of the
# kernel intervals (device busy) vs the wall span, and the sum of kernel durations
# (overlap factor).  Output: gpurun_out/<tag>_busy.txt
set -e
TAG=${1:-busy}
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kbusy -o run -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu --latency 0 --legs none > /tmp/kbusy.log 2>&1
python3 - "$R/gpurun_out/${TAG}_busy.txt" <<'PY'
import csv, glob, sys
f = glob.glob("/tmp/kbusy/**/*kernel_trace.csv", recursive=True)[0]
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in csv.DictReader(open(f))]
q = sorted(k for k in ks if "yrwi::k_" in k[2] and "k_validate" not in k[2] and "k_features" not in k[2])
t0, t1 = q[0][0], max(k[1] for k in q)
mid = t0 + (t1 - t0) // 2
w = [k for k in q if k[0] >= mid]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in w:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = max(k[1] for k in w) - w[0][0]
tot = sum(e - s for s, e, _ in w)
by = {}
for s, e, n in w: by[n] = by.get(n, 0) + (e - s)
with open(sys.argv[1], "w") as o:
    o.write("window %.3f ms  busy(union) %.3f ms (%.1f%%)  sum of kernels %.3f ms  overlap %.2f\n" % (span / 1e6, busy / 1e6, 100.0 * busy / span, tot / 1e6, tot / max(busy, 1)))
    for n, d in sorted(by.items(), key=lambda x: -x[1]): o.write("  %-40s %.3f ms\n" % (n[:40], d / 1e6))
PY
