import time, ctypes, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch
from yacy_search_server_amd import RWIIndex, RankingProfile, synth
from yacy_search_server_amd._lib import CHit, CStats
import bench
cfg = synth.preset("C2")
idx = synth.build_index(cfg)
ix = RWIIndex(0)
for t in range(cfg.n_terms):
    if idx.sizes[t]:
        ix.add(idx.hashes[t], idx.list_rows(t))
ix.build_url_ids()
qs = synth.queries(cfg, 1000, 2, 2, 0)
cq, keep = bench.build_queries(idx.hashes, qs, 100, 20741 * 86400000, RankingProfile())
hits = ix.host_array(CHit, 1000 * 100); nout = ix.host_array(ctypes.c_int32, 1000); st = CStats()
for i in range(12):
    t0 = time.perf_counter()
    t = ix.submit_raw(cq, 1000, 100, hits, nout, st)
    t1 = time.perf_counter()
    ix.wait(t)
    t2 = time.perf_counter()
    print("step %d submit %.2f ms wait %.2f ms" % (i, (t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)
t0 = time.perf_counter(); torch.cuda.synchronize(); print("sync %.2f ms" % ((time.perf_counter() - t0) * 1e3))
t0 = time.perf_counter(); torch.cuda.synchronize(); print("sync2 %.2f ms" % ((time.perf_counter() - t0) * 1e3))
