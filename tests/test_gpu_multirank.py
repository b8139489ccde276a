"""Sharded (multi-rank) libyrwi path on ONE GPU: world ranks, each a process
that owns one URL-hash shard on device 0 and talks to the others over RCCL.
This exercises yrwi_open_shard, the ShardSum all-gather + ordered combine and
the top-k all-gather merge end to end; the result must be bit-exact against
the single-container oracle.  If RCCL refuses several ranks on one device the
test is skipped (the 8-GPU path is then covered only by the driver's runs and
by tests/test_multi_gloo.py)."""

import os
import sys

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
        try:
            ix = RWIIndex(0, shard=(rank, world, uid))
        except Exception as e:  # RCCL refused several ranks on one GPU
            out_q.put((rank, "skip", str(e)))
            return
        for t in range(full.n_terms):
            if part.sizes[t]:
                ix.add(part.hashes[t], part.list_rows(t))
        qs = synth.queries(full, 24, 1, 4, 1, qseed=41)
        c5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")  # authority -> host-count exchange
        batch = [Query([part.hashes[t] for t in inc], [part.hashes[t] for t in exc], now_ms=NOW, k=100,
                       profile=(c5 if i % 2 else None)) for i, (inc, exc) in enumerate(qs)]
        got = ix.search_batch(batch)
        whole = synth.build_index(full).as_dict()
        bad = []
        for qi, (q, g) in enumerate(zip(batch, got)):
            prof = orc.profile_from(q.profile) if q.profile is not None else None
            exp = orc.search(whole, q.include, q.exclude, profile=prof, now_ms=NOW, k=100)
            if [(h.urlhash, h.score, h.tiebreak) for h in g] != exp:
                bad.append(qi)
        ix.close()
        out_q.put((rank, "ok", bad))
    except Exception as e:  # report, never hang the parent
        out_q.put((rank, "error", repr(e)))


@pytest.mark.parametrize("world", [2])
def test_sharded_query_on_one_gpu(world):
    import torch.multiprocessing as mp
    from yacy_search_server_amd import unique_id
    uid = unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, uid, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    for _ in procs:
        res.append(q.get(timeout=300))
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    if any(r[1] == "skip" for r in res):
        pytest.skip("RCCL refused %d ranks on one GPU: %s" % (world, [r[2] for r in res if r[1] == "skip"][0]))
    for rank, status, info in res:
        assert status == "ok", (rank, info)
        assert info == [], (rank, info)
