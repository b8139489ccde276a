"""Print the per-kernel table of profiles/pmc_<config>.json (after tools/pmc_summary.py)."""
import json
import sys

d = json.load(open(sys.argv[1]))
rows = sorted(d["kernels"].items(), key=lambda kv: -kv[1].get("avg_ns", 0) * kv[1].get("calls", 0))
for k, v in rows:
    if not k.startswith("k_"):
        continue
    print(f"{k:14s} calls={v.get('calls')} avg_us={v.get('avg_ns', 0) / 1e3:8.1f} "
          f"hbm_MB={(v.get('hbm_bytes_per_launch') or 0) / 1e6:8.1f}")
