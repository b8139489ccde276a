"""Collect the bench lines of the per-config runs (gpurun_out/cfg/*.json) into one
summary file under profiles/: value, ms/step, per-phase times, parity spot check,
CPU baselines.  Usage: python tools/cfg_summary.py <src_dir> <out.json>"""
import glob
import json
import os
import sys

KEEP = ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "inflight", "config", "roofline",
        "roofline_probe", "phase_ms", "parity_sample", "latency_ms", "cpu_baseline", "cpu_baseline_1thread",
        "joined_per_step", "bytes_alg_per_step")


def main(src, out):
    res = {}
    for f in sorted(glob.glob(os.path.join(src, "*.json"))):
        try:
            d = json.load(open(f))
        except (ValueError, OSError):
            continue
        res[os.path.basename(f)[:-5]] = {k: d.get(k) for k in KEEP}
    with open(out, "w") as o:
        json.dump(res, o, indent=1)
    for k, d in res.items():
        print(f"{k:12s} {d['value'] / 1e9:8.1f} G postings/s  {d['ms_per_step']:8.2f} ms/step  "
              f"parity {d['parity_sample']}  {d['config']['workload']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
