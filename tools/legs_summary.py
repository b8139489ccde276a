"""Print ms/step, isolated kernel time and per-kernel mean launch times of bench leg JSON files."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", e)
        continue
    legs = d.get("legs") or {}
    if not legs and "value" in d:
        legs = {"main": d}
    for name, L in legs.items():
        rl = L.get("roofline") or {}
        iso = (rl.get("path") or {}).get("isolated") or {}
        ks = {k: v.get("mean_launch_us") for k, v in (L.get("kernels") or {}).items() if isinstance(v, dict)}
        print(f.split("/")[-1], name, "ms/step", round(L.get("ms_per_step", 0), 3),
              "ident", (L.get("identical_batch") or {}).get("ms_per_step"),
              "iso_us", iso.get("kernel_us_per_batch"), ks)
