"""Per-step spans from a rocprofv3 kernel trace: time between consecutive k_partition
launches, and the largest idle gaps with the kernels around them."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_validate" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [int(r["Start_Timestamp"]) for r in rows if "k_partition" in r["Kernel_Name"]]
print("step spans (us):", " ".join("%.0f" % ((b - a) / 1e3) for a, b in zip(st, st[1:])))
gaps = []
for a, b in zip(rows, rows[1:]):
    g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
    gaps.append((g, a["Kernel_Name"].split("(")[0][:30], b["Kernel_Name"].split("(")[0][:30]))
gaps.sort(reverse=True)
for g, a, b in gaps[:15]:
    print("gap %9.1f us after %-30s before %s" % (g / 1e3, a, b))
