"""tools/pmc_summary.py on synthetic rocprofv3 CSVs (no GPU): a join step's
compaction is k_compact, k_compact_sum or both, pooled per step (k_scan_tiles runs
once per step) into the "compaction" entry bench.py holds against its HIP events;
k_compact_sum and k_piece_merge are keyed apart from k_compact and k_reduce."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_compaction_pooled_per_step(tmp_path):
    base = tmp_path / "prof" / "t"
    names = {"cs": "void yrwi::k_compact_sum<true>(yrwi::JoinQ const*, long const*)",
             "c": "void yrwi::k_compact<true>(yrwi::JoinQ const*, long const*)",
             "st": "yrwi::k_scan_tiles(yrwi::JoinQ const*)", "pm": "yrwi::k_piece_merge(yrwi::RankQ const*)",
             "cb": "yrwi::k_combine(yrwi::RankQ const*)"}
    # two steps: both kernels in step 1, k_compact_sum alone in step 2
    _write(str(base / "kt" / "run_kernel_stats.csv"), ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"],
           [[names["cs"], 2, 600000, 300000, 50], [names["c"], 1, 100000, 100000, 10],
            [names["st"], 2, 20000, 10000, 1], [names["pm"], 2, 50000, 25000, 2], [names["cb"], 1, 8000, 8000, 1]])
    rd = []
    wr = []
    for did, (k, b) in enumerate([("cs", 1000), ("cs", 3000), ("c", 500), ("pm", 10), ("cb", 1)]):
        rd.append([names[k], did, "TCC_EA0_RDREQ_128B_sum", b])
        wr.append([names[k], did, "TCC_EA0_WRREQ_64B_sum", b // 10])
        wr.append([names[k], did, "TCC_EA0_WRREQ_sum", b // 10])
    hdr = ["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"]
    _write(str(base / "rd" / "run_counter_collection.csv"), hdr, rd)
    _write(str(base / "wr" / "run_counter_collection.csv"), hdr, wr)
    out = tmp_path / "out"
    env = dict(os.environ, PROF_BASE=str(tmp_path / "prof"), PROF_OUT=str(out), PROF_HEAD="test")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), "t", "CX"], env=env,
                          stdout=subprocess.DEVNULL)
    d = json.load(open(out / "pmc_CX.json"))
    k = d["kernels"]
    assert {"k_compact_sum", "k_compact", "k_piece_merge", "k_scan_tiles"} <= set(k)
    c = k["compaction"]
    assert c["calls"] == 2 and c["pooled"] == ["k_compact", "k_compact_sum"]
    assert c["avg_ns"] == (600000 + 100000) / 2
    # bytes per step: every dispatch's reads (128 B each) + writes (64 B each), over the two steps
    total = sum(128 * b + 64 * (b // 10) for b in (1000, 3000, 500))
    assert abs(c["hbm_bytes_per_launch"] - total / 2) < 1e-6
    assert d["compaction_avg_ns"] == c["avg_ns"]
