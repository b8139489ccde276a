"""Sharded (multi-rank) libyrwi path on ONE GPU: world ranks, each a process
that owns one URL-hash shard on device 0.  RCCL refuses several ranks on one
device, so the ranks' device collectives (ShardSum all-gather, authority
host-count exchange, top-k all-gather) run host-staged through the node's
shared memory (yrwi_coll.cpp): "auto" (an RCCL unique id) finds through the
mailbox that the ranks' PCI bus ids are equal and never tries RCCL; "staged"
names the transport in the group id (YRWI-HOSTSTAGE).  Each rank's
yrwi_shard_info must say host-staged.  The list-size
planning goes through the host mailbox as on the 8-GPU node.  This runs
yrwi_open_shard, global-size planning, the ordered combine, the host-count
exchange and the top-k merge of libyrwi across processes; the result must be
bit-exact against the single-container oracle (authority profile included)."""

import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NOW = 20741 * 86400000 + 31337


def _rank_main(rank, world, uid, out_q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle as orc
        from yacy_search_server_amd import Query, RankingProfile, RWIIndex, synth
        full = synth.preset("small")
        part = synth.build_index(full.shard(rank, world))
        ix = RWIIndex(0, shard=(rank, world, uid))
        info = ix.shard_info()
        for t in range(full.n_terms):
            if part.sizes[t]:
                ix.add(part.hashes[t], part.list_rows(t))
        qs = synth.queries(full, 36, 1, 4, 1, qseed=41)
        c5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")  # authority -> host-count exchange
        batch = [Query([part.hashes[t] for t in inc], [part.hashes[t] for t in exc], now_ms=NOW, k=100,
                       profile=(c5 if i % 2 else None)) for i, (inc, exc) in enumerate(qs)]
        # one synchronous batch (split over the lanes), then two in flight on different lanes
        got = ix.search_batch(batch[:12])
        p1 = ix.submit(batch[12:24])
        p2 = ix.submit(batch[24:])
        got += p1.result() + p2.result()
        whole = synth.build_index(full).as_dict()
        bad = []
        for qi, (q, g) in enumerate(zip(batch, got)):
            prof = orc.profile_from(q.profile) if q.profile is not None else None
            exp = orc.search(whole, q.include, q.exclude, profile=prof, now_ms=NOW, k=100)
            if [(h.urlhash, h.score, h.tiebreak) for h in g] != exp:
                bad.append(qi)
        ix.close()
        out_q.put((rank, "ok", (bad, info)))
    except Exception as e:  # report, never hang the parent
        out_q.put((rank, "error", repr(e)))


@pytest.mark.parametrize("world,transport", [(2, "auto"), (2, "staged"), (4, "staged")])
def test_sharded_query_on_one_gpu(world, transport, monkeypatch):
    import queue
    import time
    import torch.multiprocessing as mp
    from yacy_search_server_amd import unique_id
    # a rank that fails must not leave its peers waiting out the default 300 s
    monkeypatch.setenv("YRWI_HOSTX_TIMEOUT_S", "30")
    uid = unique_id() if transport == "auto" else b"YRWI-HOSTSTAGE\0" + os.urandom(113)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, uid, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    deadline = time.time() + 90
    try:
        for _ in procs:
            res.append(q.get(timeout=max(1.0, deadline - time.time())))
    except queue.Empty:
        pass
    for p in procs:
        p.join(timeout=max(1.0, deadline + 10 - time.time()))
        if p.is_alive():
            p.kill()
    assert len(res) == world, ("ranks that never reported", res)
    for rank, status, info in res:
        assert status == "ok", (rank, info)
        bad, tinfo = info
        assert bad == [], (rank, bad)
        assert tinfo["transport"] == "host-staged", tinfo
        assert tinfo["rank"] == rank and tinfo["world"] == world and tinfo["rccl_ranks"] == 0, tinfo
        assert tinfo["device_peers"] == world - 1 and tinfo["mailbox"] == 1, tinfo


def test_rccl_self_world1(monkeypatch):
    """The sharded protocol over a REAL 1-rank RCCL communicator on this GPU
    (YRWI_COLL_SELF=1, yrwi_open_shard with world 1): global-size planning goes
    through the device all-gather (no host mailbox at world 1), then the ShardSum
    all-gather, the authority host-count exchange (grouped ncclSend / ncclRecv to
    self and the max all-reduce), the flag-count all-reduce and the top-k
    all-gather + shard merge -- every RCCL call site of yrwi_coll.cpp with the
    production counts, types and streams.  Bit-exact against the oracle."""
    monkeypatch.setenv("YRWI_COLL_SELF", "1")
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import java_literal as jl
    import oracle as orc
    from yacy_search_server_amd import Query, QueryFilter, RankingProfile, RWIIndex, synth, unique_id
    full = synth.preset("small")
    idx = synth.build_index(full)
    ix = RWIIndex(0, shard=(0, 1, unique_id()))
    try:
        info = ix.shard_info()
        assert info["transport"] == "rccl" and info["rccl_ranks"] == 1 and info["world"] == 1, info
        assert info["lanes_own_comm"] == info["lanes"] >= 1, info
        for t in range(full.n_terms):
            if idx.sizes[t]:
                ix.add(idx.hashes[t], idx.list_rows(t))
        maps = open("/proc/self/maps").read()
        assert "librccl" in maps, "RCCL is not mapped into the process"
        qs = synth.queries(full, 40, 1, 4, 1, qseed=43)
        c5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")  # authority -> send/recv to self
        batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], now_ms=NOW, k=100,
                       profile=(c5 if i % 2 else None)) for i, (inc, exc) in enumerate(qs)]
        # two batches in flight on different lanes: the collective turn orders their RCCL calls
        p1 = ix.submit(batch[:20])
        p2 = ix.submit(batch[20:])
        got = p1.result() + p2.result()
        whole = idx.as_dict()
        for qi, (q, g) in enumerate(zip(batch, got)):
            prof = orc.profile_from(q.profile) if q.profile is not None else None
            exp = orc.search(whole, q.include, q.exclude, profile=prof, now_ms=NOW, k=100)
            assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp, qi
        # flag counts: the all-reduce of the counters
        big = [int(t) for t in np.argsort(-idx.sizes)[:2]]
        lit = {h: [bytes(x) for x in rows] for h, rows in whole.items()}
        for kw in (dict(constraint=b"\0\0\x10\x01"), dict(skip_double_dom=True)):
            q = Query([idx.hashes[t] for t in big], [], now_ms=NOW, k=50, filter=QueryFilter(**kw))
            (g,) = ix.search_batch([q])
            lf = jl.QueryFilter(**kw)
            e = jl.search(lit, q.include, q.exclude, jl.RankingProfile(), "en", now_ms=NOW, k=50, filt=lf)
            assert [(h.urlhash, h.score) for h in g] == e, kw
            assert q.filter.flagcount == lf.flagcount, kw
    finally:
        ix.close()
