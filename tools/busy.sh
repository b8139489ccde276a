#!/bin/bash
# GPU busy fraction of the default (four batches in flight) C2 bench: kernel trace of a
# bench run, then over the query kernels of the middle 60% of the run (timed region): union of the
# kernel intervals (device busy) vs the wall span, and the sum of kernel durations
# (overlap factor).  Output: gpurun_out/<tag>_busy.txt
set -e
TAG=${1:-busy}
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kbusy -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu --latency 0 --legs none > /tmp/kbusy.log 2>&1
python3 - "$R/gpurun_out/${TAG}_busy.txt" <<'PY'
import csv, glob, sys
f = glob.glob("/tmp/kbusy/**/*kernel_trace.csv", recursive=True)[0]
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in csv.DictReader(open(f))]
q = sorted(k for k in ks if "yrwi::k_" in k[2] and "k_validate" not in k[2] and "k_features" not in k[2])
t0, t1 = q[0][0], max(k[1] for k in q)
lo, hi = t0 + (t1 - t0) // 5, t0 + 4 * (t1 - t0) // 5  # inside the timed region (200 steps)
w = [k for k in q if lo <= k[0] < hi]
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
# idle gaps of the device (no kernel running), by length, with the kernel that ends before each
gaps = []
end = w[0][1]
last = w[0][2]
for s, e, n in w[1:]:
    if s > end:
        gaps.append((s - end, last, n))
    if e > end:
        end, last = e, n
hist = {}
for g, a, b in gaps:
    key = "<5us" if g < 5000 else "<20us" if g < 20000 else "<50us" if g < 50000 else "<100us" if g < 100000 else ">=100us"
    c = hist.setdefault(key, [0, 0])
    c[0] += 1
    c[1] += g
pairs = {}
for g, a, b in gaps:
    k = a.split("::")[-1][:16] + " -> " + b.split("::")[-1][:16]
    pairs[k] = pairs.get(k, 0) + g
with open(sys.argv[1], "w") as o:
    o.write("idle gaps: " + "  ".join("%s: %d (%.3f ms)" % (k, v[0], v[1] / 1e6) for k, v in sorted(hist.items())) + "\n")
    for k, v in sorted(pairs.items(), key=lambda x: -x[1])[:10]: o.write("  gap after/before %-40s %.3f ms\n" % (k, v / 1e6))
    o.write("window %.3f ms  busy(union) %.3f ms (%.1f%%)  sum of kernels %.3f ms  overlap %.2f\n" % (span / 1e6, busy / 1e6, 100.0 * busy / span, tot / 1e6, tot / max(busy, 1)))
    for n, d in sorted(by.items(), key=lambda x: -x[1]): o.write("  %-40s %.3f ms\n" % (n[:40], d / 1e6))
PY
