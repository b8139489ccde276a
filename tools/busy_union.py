"""GPU occupancy of bench.py's timed region from a rocprofv3 kernel trace (run the
bench with YRWI_BENCH_GAP_MS=50: idle gaps of that length bracket the region).
Prints the region's span, the union of kernel intervals (the GPU busy with at
least one kernel), the time-weighted mean number of kernels running at once,
and per kernel its share of the region."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].split("::")[-1]) for r in rows)
gap_ns = float(sys.argv[2]) * 1e6 * 0.8 if len(sys.argv) > 2 else 40e6
# the region: the stretch between two consecutive idle gaps longer than gap_ns
# that holds the most k_compact dispatches (the index build has gaps of its own)
ends, cuts = 0, []
for s, e, n in iv:
    if ends and s - ends > gap_ns:
        cuts.append((ends, s))
    ends = max(ends, e)
if len(cuts) < 2:
    sys.exit("no bracketing gaps found: %d" % len(cuts))
best = max(range(len(cuts) - 1),
           key=lambda i: sum(1 for s, e, n in iv if s >= cuts[i][1] and e <= cuts[i + 1][0] and n.startswith("k_compact")))
r0, r1 = cuts[best][1], cuts[best + 1][0]
sel = [(s, e, n) for s, e, n in iv if s >= r0 and e <= r1]
span = r1 - r0
# union and concurrency
ev = sorted([(s, 1) for s, _, _ in sel] + [(e, -1) for _, e, _ in sel])
busy = conc = 0
cur, last = 0, r0
for t, d in ev:
    if cur > 0:
        busy += t - last
        conc += cur * (t - last)
    cur += d
    last = t
per = defaultdict(int)
for s, e, n in sel:
    per[n] += e - s
print(f"region {span / 1e3:.1f} us, kernels {len(sel)}, GPU busy (union) {busy / span:.3f}, "
      f"mean kernels at once while busy {conc / max(busy, 1):.2f}")
for n, t in sorted(per.items(), key=lambda x: -x[1])[:16]:
    print(f"  {n:28s} {t / 1e3:9.1f} us summed  ({t / span:.2f} of the region)")
