"""Summarise a rocprofv3 --stats kernel_stats.csv: name, calls, average, total."""
import csv
import glob
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"([^(<]*(?:<[^>]*>)?)", name)
    return (m.group(1) if m else name)[:60]


def main(src_dir: str, out: str) -> None:
    f = glob.glob(src_dir + "/**/*kernel_stats.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    with open(out, "w") as o:
        for r in rows:
            o.write("%-60s %6s %10.1f us %10.2f ms total\n" % (short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3,
                                                            float(r["TotalDurationNs"]) / 1e6))


def dispatches(src_dir: str, kernel: str) -> list:
    """per-dispatch durations (us) of one kernel from kernel_trace.csv, in dispatch order"""
    f = glob.glob(src_dir + "/**/*kernel_trace.csv", recursive=True)[0]
    out = []
    for r in csv.DictReader(open(f)):
        if kernel in r["Kernel_Name"]:
            out.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return [d for _, d in sorted(out)]


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
    for k in sys.argv[3:]:
        with open(sys.argv[2], "a") as o:
            o.write("%s per dispatch (us): %s\n" % (k, " ".join("%.1f" % d for d in dispatches(sys.argv[1], k))))

