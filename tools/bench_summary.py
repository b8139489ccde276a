"""One line per bench config of a bench JSON file: ms/step, postings/s, dominant kernel, fractions, parity."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rows = [("C2", d)] + list((d.get("legs") or {}).items())
for n, L in rows:
    if "ms_per_step" not in L:
        print(n, L)
        continue
    r = L["roofline"]
    ps = L.get("parity_sample") or {}
    print(f"{n:10s} {L['ms_per_step']:.3f} ms  {L['value']:.3g} p/s  {r.get('kernel')} frac {r.get('frac')} "
          f"hbm {r.get('hbm_frac')}  parity {ps.get('queries_checked')}/{ps.get('mismatches')}  "
          f"phase {L.get('phase_ms')}")
cb = d.get("cpu_baseline") or {}
print("cpu", cb.get("value"), cb.get("cores"), cb.get("sample"))
