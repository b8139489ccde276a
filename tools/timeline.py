"""Timeline of one bench step from a rocprofv3 kernel trace: kernels in dispatch
order with their start offset, duration and the idle gap before each."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "k_validate" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last step: from the last k_partition back to its preceding k_emit
starts = [i for i, r in enumerate(rows) if "k_partition" in r["Kernel_Name"]]
i0 = starts[-2] if len(starts) > 1 else starts[-1]
i1 = starts[-1]
t0 = int(rows[i0]["Start_Timestamp"])
prev_end = None
busy = 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("yrwi::", "")[:28]
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} us  {name:28s} dur {(e - s) / 1e3:8.1f}  gap {gap:8.1f}  grid {r['Grid_Size_X']}")
    prev_end = e
print(f"step span {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us")
