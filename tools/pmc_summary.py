"""Summarise rocprofv3 CSV output of tools/profile_gpu.sh into profiles/.

profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (copied)
profiles/pmc_<config>.json        per-kernel mean duration and HBM bytes per launch
HBM bytes per dispatch = read requests leaving L2 by size (32 TCC_EA0_RDREQ_32B + 64
TCC_EA0_RDREQ_64B + 128 TCC_EA0_RDREQ_128B) + write requests (64 TCC_EA0_WRREQ_64B + 32
(TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B)); TCC_EA0_RDREQ_DRAM = the reads that reached DRAM
(the rest were served by the Infinity Cache).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(pattern):
    return sorted(glob.glob(pattern, recursive=True))


def short(name):
    # k_probe<LONG, MARK>: the exclusion steps' dispatches (MARK) are keyed apart from the include steps'
    if "k_probe<" in name and "k_probe_part" not in name:
        args = name.split("k_probe<", 1)[1].split(">", 1)[0].replace(" ", "").split(",")
        return "k_probe_excl" if len(args) > 1 and args[1] in ("true", "1") else "k_probe"
    if "k_probeILb" in name:
        return "k_probe_excl" if "ELb1E" in name.split("k_probeILb", 1)[1][:8] else "k_probe"
    for k in ("k_chain_part", "k_chain", "k_join", "k_probe_part", "k_probe", "k_partition", "k_topq", "k_scan_tiles", "k_scan_bounds",
              "k_compact_sum", "k_compact", "k_piece_merge", "k_reduce", "k_shard_fin", "k_combine", "k_order_hist", "k_order_scatter", "k_copy_in",
              "k_score_all", "k_score_full", "k_score", "k_merge", "k_emit", "k_validate", "k_features", "k_feat_rows"):
        if k + "E" in name or name.endswith(k) or (k + "I") in name or k in name:
            return k
    return name[:40]


def counters(path):
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for f in find(os.path.join(path, "**", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            did = row.get("Dispatch_Id") or row.get("Correlation_Id")
            per[k][row.get("Counter_Name")] += float(row.get("Counter_Value", 0))
            n[k].add(did)
    return per, {k: len(v) for k, v in n.items()}


def main(tag, config):
    # PROF_BASE: where tools/profile_gpu.sh left the raw output; PROF_OUT: where the
    # summaries go (on the GPU box: a directory under gpurun_out/, copied into profiles/)
    base = os.path.join(os.environ.get("PROF_BASE", os.path.join(ROOT, "gpurun_out", "prof")), tag)
    pout = os.environ.get("PROF_OUT", os.path.join(ROOT, "profiles"))
    os.makedirs(pout, exist_ok=True)
    stats = find(os.path.join(base, "kt", "**", "*kernel_stats.csv"))
    out = {"tag": tag, "config": config, "kernels": {}}
    if stats:
        shutil.copy(stats[0], os.path.join(pout, f"{tag}_kernel_stats.csv"))
        for row in csv.DictReader(open(stats[0])):
            k = short(row["Name"])  # template instances (k_probe<true> / <false>) pool into one entry
            d = out["kernels"].setdefault(k, {"calls": 0, "total_ns": 0.0, "pct": 0.0})
            d["calls"] += int(row["Calls"])
            d["total_ns"] += float(row["AverageNs"]) * int(row["Calls"])
            d["avg_ns"] = d["total_ns"] / d["calls"]
            d["pct"] += float(row.get("Percentage", 0))
    # per-dispatch durations of the query path's kernels (the kernel trace of the same run)
    traces = find(os.path.join(base, "kt", "**", "*kernel_trace.csv"))
    if traces:
        with open(os.path.join(pout, f"{tag}_dispatches.csv"), "w") as o:
            o.write("kernel,grid,duration_ns\n")
            for row in csv.DictReader(open(traces[0])):
                k = short(row.get("Kernel_Name", ""))
                if k.startswith("k_") and k not in ("k_validate", "k_features"):
                    g = row.get("Grid_Size_X") or row.get("Grid_Size") or 0
                    o.write(f"{k},{g},{int(row['End_Timestamp']) - int(row['Start_Timestamp'])}\n")
    rd, nr = counters(os.path.join(base, "rd"))
    wr, nw = counters(os.path.join(base, "wr"))
    for k in set(rd) | set(wr):
        d = out["kernels"].setdefault(k, {})
        if k in rd and nr.get(k):
            c = rd[k]
            rb = 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) + \
                128 * c.get("TCC_EA0_RDREQ_128B_sum", 0)
            d["read_bytes_per_launch"] = rb / nr[k]
            d["read_requests_dram_per_launch"] = c.get("TCC_EA0_RDREQ_DRAM_sum", 0) / nr[k]
        if k in wr and nw.get(k):
            c = wr[k]
            w64 = c.get("TCC_EA0_WRREQ_64B_sum", 0)
            d["write_bytes_per_launch"] = (64 * w64 + 32 * (c.get("TCC_EA0_WRREQ_sum", 0) - w64)) / nw[k]
        if "read_bytes_per_launch" in d and "write_bytes_per_launch" in d:
            d["hbm_bytes_per_launch"] = d["read_bytes_per_launch"] + d["write_bytes_per_launch"]
    # one batch's HBM traffic: every kernel of the query path, per launch x launches per batch
    # (k_combine runs once per batch pass); index build, uploads and fills excluded
    path = ("k_partition", "k_probe_part", "k_scan_bounds", "k_order_hist", "k_order_scatter", "k_join", "k_probe",
            "k_probe_excl", "k_chain_part", "k_chain", "k_scan_tiles", "k_compact", "k_compact_sum", "k_piece_merge",
            "k_reduce", "k_shard_fin", "k_combine", "k_score", "k_score_full", "k_topq", "k_emit")
    # a join step's compaction (launch_compact) is k_compact, k_compact_sum (the jobs
    # with normalisation pieces) or both: per step (k_scan_tiles runs once per step)
    # they pool into "compaction", the figure bench.py holds against its HIP events
    steps = out["kernels"].get("k_scan_tiles", {}).get("calls")
    parts = [out["kernels"][k] for k in ("k_compact", "k_compact_sum") if k in out["kernels"]]
    if steps and parts:
        c = {"calls": steps, "total_ns": sum(p.get("total_ns", 0.0) for p in parts),
             "pooled": [k for k in ("k_compact", "k_compact_sum") if k in out["kernels"]]}
        c["avg_ns"] = c["total_ns"] / steps
        if all("hbm_bytes_per_launch" in p and p.get("calls") for p in parts):
            c["hbm_bytes_per_launch"] = sum(p["hbm_bytes_per_launch"] * p["calls"] for p in parts) / steps
        if all("read_requests_dram_per_launch" in p and p.get("calls") for p in parts):
            c["read_requests_dram_per_launch"] = sum(p["read_requests_dram_per_launch"] * p["calls"]
                                                     for p in parts) / steps
        out["kernels"]["compaction"] = c
    nb = out["kernels"].get("k_combine", {}).get("calls")
    if nb:
        tot = 0.0
        for k in path:
            kd = out["kernels"].get(k, {})
            if kd.get("hbm_bytes_per_launch") and kd.get("calls"):
                tot += kd["hbm_bytes_per_launch"] * kd["calls"]
        out["path_hbm_bytes_per_batch"] = tot / nb
        out["batches_profiled"] = nb
    # the build measured: the same (head, src) pair bench.py stamps on its line (the
    # GPU box has no .git: head comes from PROF_HEAD or the REVISION file)
    sys.path.insert(0, ROOT)
    from bench import source_identity
    ident = source_identity()
    out["head"] = os.environ.get("PROF_HEAD") or ident["head"]
    out["src"] = ident["src"]
    for name in ("compaction", "k_compact", "k_compact_sum", "k_join", "k_probe", "k_probe_excl", "k_chain", "k_reduce",
                 "k_piece_merge", "k_score"):
        kd = out["kernels"].get(name, {})
        out[name + "_hbm_bytes_per_launch"] = kd.get("hbm_bytes_per_launch")
        out[name + "_avg_ns"] = kd.get("avg_ns")
    for log in ("kt.log", "rd.log", "wr.log"):
        p = os.path.join(base, log)
        if os.path.exists(p):
            for line in open(p):
                if line.startswith("{") and '"metric"' in line:
                    out.setdefault("bench_lines", {})[log] = json.loads(line)
    with open(os.path.join(pout, f"pmc_{config}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "bench_lines"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01", sys.argv[2] if len(sys.argv) > 2 else "C2")
