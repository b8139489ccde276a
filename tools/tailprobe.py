"""Which queries set the per-batch kernel times: runs (a) the single largest C2 query,
(b) the C2 batch, (c) the C2 batch without queries whose both terms are among the 10
largest lists, 4 times each, in that order (read the per-dispatch durations from a
rocprofv3 kernel trace with tools/kstats_summary.py)."""
import ctypes
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from yacy_search_server_amd import RWIIndex, RankingProfile, synth  # noqa: E402
from yacy_search_server_amd._lib import CHit, CStats  # noqa: E402

cfg = synth.preset("C2")
idx = synth.build_index(cfg)
ix = RWIIndex(0)
for t in range(cfg.n_terms):
    if idx.sizes[t]:
        ix.add(idx.hashes[t], idx.list_rows(t))
ix.build_url_ids()
qs = synth.queries(cfg, 1000, 2, 2, 0)
big = set(int(t) for t in sorted(range(cfg.n_terms), key=lambda t: -idx.sizes[t])[:10])
top2 = sorted(range(cfg.n_terms), key=lambda t: -idx.sizes[t])[:2]
small = [q for q in qs if not (q[0][0] in big and q[0][1] in big)]
now = 20741 * 86400000
for name, batch in (("largest", [([int(top2[0]), int(top2[1])], [])]), ("c2", qs), ("small", small)):
    cq, keep = bench.build_queries(idx.hashes, batch, 100, now, RankingProfile())
    hits = ix.host_array(CHit, len(batch) * 100)
    nout = ix.host_array(ctypes.c_int32, len(batch))
    for i in range(4):
        ix.wait(ix.submit_raw(cq, len(batch), 100, hits, nout, CStats()))
    print(name, len(batch), "queries", flush=True)
ix.close()
