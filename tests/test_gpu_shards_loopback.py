"""Sharded libyrwi path on ONE GPU through the in-process loopback transport.

RCCL refuses two ranks on one device (tests/test_gpu_multirank.py skips on a
one-GPU box), so these tests open `world` shard contexts in one process, each
driven by its own thread, joined by a loopback group id (yrwi_coll.cpp).  Every
step of the sharded path runs as in production -- vertical-DHT url-hash shards,
ShardSum all-gather + ordered combine, the authority host-count owner exchange,
flag-count all-reduce, the cross-shard top-k merge and the doubledom pull -- only
the transport is a device-to-device copy instead of RCCL.  Results must be
bit-exact against the single-container oracle."""

import os
import threading

import numpy as np
import pytest

import java_literal as jl
import oracle as orc
from yacy_search_server_amd import Query, QueryFilter, RankingProfile, RWIIndex, synth

pytestmark = pytest.mark.gpu

NOW = 20741 * 86400000 + 31337


def _loop_id():
    return b"YRWI-LOOPBACK\0" + os.urandom(114)


def _run_shards(full, world, make_batch):
    """Open `world` shards of `full` on GPU 0, run make_batch(part) on each from its
    own thread; returns per-rank (batch, results)."""
    uid = _loop_id()
    parts = [synth.build_index(full.shard(r, world)) for r in range(world)]
    ixs = [None] * world
    out = [None] * world
    errs = []

    def opener(r):
        try:
            ixs[r] = RWIIndex(0, shard=(r, world, uid))
            p = parts[r]
            for t in range(full.n_terms):
                if p.sizes[t]:
                    ixs[r].add(p.hashes[t], p.list_rows(t))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    def runner(r):
        try:
            batch = make_batch(parts[r])
            out[r] = (batch, ixs[r].search_batch(batch))
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))

    for fn in (opener, runner):
        ths = [threading.Thread(target=fn, args=(r,)) for r in range(world)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=300)
        assert not errs, errs
    for ix in ixs:
        ix.close()
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_loopback_shards_bit_exact(world):
    full = synth.preset("small")
    qs = synth.queries(full, 24, 1, 4, 1, qseed=41)
    c5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")  # authority -> host-count exchange

    def make_batch(part):
        return [Query([part.hashes[t] for t in inc], [part.hashes[t] for t in exc], now_ms=NOW, k=100,
                      profile=(c5 if i % 2 else None)) for i, (inc, exc) in enumerate(qs)]

    res = _run_shards(full, world, make_batch)
    whole = synth.build_index(full).as_dict()
    for r, (batch, got) in enumerate(res):
        for qi, (q, g) in enumerate(zip(batch, got)):
            prof = orc.profile_from(q.profile) if q.profile is not None else None
            exp = orc.search(whole, q.include, q.exclude, profile=prof, now_ms=NOW, k=100)
            assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp, (r, qi)


def test_loopback_shards_filters_and_doubledom():
    world = 2
    full = synth.preset("tiny")
    idx = synth.build_index(full)
    big = [int(t) for t in np.argsort(-idx.sizes)[:3]]
    rng = np.random.default_rng(5)
    hosts = sorted({bytes(r[6:12]) for r in idx.rows[rng.integers(0, len(idx.rows), 100)]})
    kws = [dict(constraint=b"\0\0\x10\x01"), dict(language="de"), dict(siteexcludes=hosts[:30]),
           dict(skip_double_dom=True), dict(skip_double_dom=True, contentdom=1)]
    queries = [([big[0]], []), ([big[1]], [big[2]]), ([big[0], big[2]], [])]
    cases = [(inc, exc, kw, k) for (inc, exc) in queries for kw in kws for k in (10, 100)]

    def make_batch(part):  # every rank gets its own filter objects (flag counts come back per rank)
        return [Query([part.hashes[t] for t in inc], [part.hashes[t] for t in exc], now_ms=NOW, k=k,
                      filter=QueryFilter(**kw)) for (inc, exc, kw, k) in cases]

    res = _run_shards(full, world, make_batch)
    lit = {h: [bytes(x) for x in rows] for h, rows in idx.as_dict().items()}
    for r, (batch, got) in enumerate(res):
        for (inc, exc, kw, k), q, g in zip(cases, batch, got):
            lf = jl.QueryFilter(**kw)
            e = jl.search(lit, q.include, q.exclude, jl.RankingProfile(), "en", now_ms=NOW, k=k, filt=lf)
            assert [(h.urlhash, h.score) for h in g] == e, (r, kw, k)
            assert q.filter.flagcount == lf.flagcount, (r, kw, k)


def _run_parts(parts, world, fn):
    """parts: per-rank {term hash: rows}; fn(rank, RWIIndex) runs on every rank's own
    thread (the same call sequence on every rank); returns the per-rank results."""
    uid = _loop_id()
    ixs = [None] * world
    out = [None] * world
    errs = []

    def opener(r):
        try:
            ixs[r] = RWIIndex(0, shard=(r, world, uid))
            for h, rows in parts[r].items():
                ixs[r].add(h, rows)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    def runner(r):
        try:
            out[r] = fn(r, ixs[r])
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))

    for f in (opener, runner):
        ths = [threading.Thread(target=f, args=(r,)) for r in range(world)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=300)
        assert not errs, errs
    for ix in ixs:
        ix.close()
    return out


def _flip_band_queries(full, whole, parts, nq, seed):
    """Queries whose result a shard-local plan would get wrong (the J2/J3 decisions
    flip on local sizes), found with the oracle, plus a few ordinary ones."""
    import shard_fold as sf
    flip, plain = [], []
    for nex in (0, 1, 2):
        for inc, exc in synth.queries(full, nq, 2, 3, nex, qseed=seed + nex):
            ih = [synth.term_hash(full, t) for t in inc]
            eh = [synth.term_hash(full, t) for t in exc]
            ref = orc.term_search(whole, ih, eh, 2147483647, NOW)
            loc = [np.asarray(x).reshape(-1, 40) for x in sf.sharded_term_search(parts, ih, eh, 2147483647, NOW, "local")]
            same = np.array_equal(np.concatenate(loc) if loc else np.zeros((0, 40), np.uint8), ref)
            (plain if same else flip).append((ih, eh))
    return flip, plain[:8]


@pytest.mark.parametrize("world", [2, 8])
def test_loopback_flip_band_global_planning(world):
    """Sharded planning on GLOBAL list sizes (J1 existence, J2 fold order, J3 dispatch of
    every step): the queries that shard-local planning gets wrong are bit-exact, both the
    joined containers (yrwi_join_exclude per shard, concatenated in shard order) and the
    ranked top-100."""
    full = synth.preset("small")
    whole = synth.build_index(full).as_dict()
    parts = [synth.build_index(full.shard(r, world)).as_dict() for r in range(world)]
    flip, plain = _flip_band_queries(full, whole, parts, 300, 7)
    assert flip, "no query in the dispatch flip band"
    cases = flip + plain

    def fn(r, ix):
        rows = [ix.term_search(ih, eh, now_ms=NOW) for ih, eh in cases]
        hits = ix.search_batch([Query(ih, eh, now_ms=NOW, k=100) for ih, eh in cases])
        return rows, hits

    res = _run_parts(parts, world, fn)
    for qi, (ih, eh) in enumerate(cases):
        ref = orc.term_search(whole, ih, eh, 2147483647, NOW)
        got = np.concatenate([res[r][0][qi].reshape(-1, 40) for r in range(world)])
        assert np.array_equal(got, ref), ("join", qi, qi < len(flip))
        exp = orc.search(whole, ih, eh, now_ms=NOW, k=100)
        for r in range(world):
            assert [(h.urlhash, h.score, h.tiebreak) for h in res[r][1][qi]] == exp, ("top-k", r, qi)


def test_loopback_exclude_term_absent_from_a_shard():
    """Two exclude terms, one of them held by a single shard: exclusion stays on for
    every shard (J1 is decided on global sizes); a globally absent exclude term turns
    all exclusion off on every shard."""
    world = 8
    full = synth.preset("small")
    whole = synth.build_index(full).as_dict()
    parts = [synth.build_index(full.shard(r, world)).as_dict() for r in range(world)]
    sizes = synth.counts(full)
    big = [int(t) for t in np.argsort(-sizes)[:3]]
    hs = [synth.term_hash(full, t) for t in big]
    rare = b"rareTERMxxxA"
    rows = parts[3][hs[0]][::3].copy()
    whole[rare] = rows
    parts[3][rare] = rows
    ih = [hs[0], hs[1]]
    cases = [(ih, [rare, hs[2]]), (ih, [rare]), (ih, [b"AAAAAAAAAAAA", hs[2]]), ([hs[0], hs[2]], [rare])]

    def fn(r, ix):
        return ix.search_batch([Query(i, e, now_ms=NOW, k=100) for i, e in cases])

    res = _run_parts(parts, world, fn)
    for qi, (i, e) in enumerate(cases):
        exp = orc.search(whole, i, e, now_ms=NOW, k=100)
        for r in range(world):
            assert [(h.urlhash, h.score, h.tiebreak) for h in res[r][qi]] == exp, (r, qi)


@pytest.mark.parametrize("world", [2, 8])
def test_loopback_async_batches_in_flight(world):
    """Sharded contexts run two lanes: several submitted batches per rank are in
    flight at once, each lane with its own group, and the batch parts enqueue
    their collectives in submission order (CollTurn).  Batches of different
    sizes and shapes (3-4 terms: fold-step size exchanges; authority profile:
    host-count exchange; an empty batch) must all come back bit-exact."""
    full = synth.preset("small")
    whole_ix = synth.build_index(full)
    whole, H = whole_ix.as_dict(), whole_ix.hashes
    c5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")
    sets = [synth.queries(full, n, 1, 4, 1, qseed=90 + i) if n else [] for i, n in enumerate([12, 5, 0, 20, 9, 3])]

    def prof(i, j):
        return c5 if (i + j) % 3 == 0 else None

    def fn(r, ix):
        pend = [ix.submit([Query([H[t] for t in inc], [H[t] for t in exc], now_ms=NOW, k=100, profile=prof(i, j))
                           for j, (inc, exc) in enumerate(qs)]) for i, qs in enumerate(sets)]
        return [p.result() for p in pend]

    parts = [synth.build_index(full.shard(r, world)).as_dict() for r in range(world)]
    res = _run_parts(parts, world, fn)
    for i, qs in enumerate(sets):
        exp = [orc.search(whole, [H[t] for t in inc], [H[t] for t in exc],
                          profile=(orc.profile_from(prof(i, j)) if prof(i, j) else None), now_ms=NOW, k=100)
               for j, (inc, exc) in enumerate(qs)]
        for r in range(world):
            got = res[r][i]
            assert len(got) == len(qs), (r, i)
            for j, g in enumerate(got):
                assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp[j], (r, i, j)


@pytest.mark.parametrize("hostx", [1, 0])
@pytest.mark.parametrize("world", [2, 8])
def test_loopback_many_batches_in_flight(world, hostx, monkeypatch):
    """Stress of the sharded lanes: 40 submitted batches per rank (more than the
    lanes and the mailbox's slot window, so lanes and slots are reused while
    other batches still run), sizes 1-30 queries with 1-4 include terms, one
    exclude term in every third batch, the authority profile in every fifth.
    hostx = 0: no shared-memory mailbox, the planning sizes go through the device
    all-gather under the collective turn.  Every batch must come back bit-exact
    and nothing may hang."""
    if not hostx:
        monkeypatch.setenv("YRWI_NO_HOSTX", "1")
    full = synth.preset("tiny")
    whole_ix = synth.build_index(full)
    whole, H = whole_ix.as_dict(), whole_ix.hashes
    c5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")
    rng = np.random.default_rng(7)
    sets = [synth.queries(full, int(rng.integers(1, 31)), 1, 4, 1 if i % 3 == 0 else 0, qseed=500 + i)
            for i in range(40)]

    def prof(i):
        return c5 if i % 5 == 0 else None

    def fn(r, ix):
        pend = [ix.submit([Query([H[t] for t in inc], [H[t] for t in exc], now_ms=NOW, k=50, profile=prof(i))
                           for inc, exc in qs]) for i, qs in enumerate(sets)]
        return [p.result() for p in pend]

    parts = [synth.build_index(full.shard(r, world)).as_dict() for r in range(world)]
    res = _run_parts(parts, world, fn)
    for i, qs in enumerate(sets):
        exp = [orc.search(whole, [H[t] for t in inc], [H[t] for t in exc],
                          profile=(orc.profile_from(prof(i)) if prof(i) else None), now_ms=NOW, k=50)
               for inc, exc in qs]
        for r in range(world):
            assert [[(h.urlhash, h.score, h.tiebreak) for h in g] for g in res[r][i]] == exp, (r, i)


@pytest.mark.parametrize("world", [2, 8])
def test_loopback_count_first_four_terms(world, monkeypatch):
    """4-term chained folds counted first (YRWI_CHAIN_CF=2 forces it; J2 puts the
    int-wrapped big lists first in C4's real queries): lists 0..2 with url-id
    bitmaps count |list 0 x list 1| and |list 0 x list 1 x list 2| by popcounts and
    the chain starts from list 3.  Whether every shard has those bitmaps is decided
    in the planning exchange (Plan::inc_allbm), so all ranks take the same fold;
    the counts are summed over the shards.  Bit-exact against the oracle, with the
    authority profile and an exclude term in some queries."""
    monkeypatch.setenv("YRWI_CHAIN_CF", "2")
    full = synth.preset("small" if world == 2 else "C1")  # big lists hold >= 4096 postings on every shard
    whole_ix = synth.build_index(full)
    whole, H = whole_ix.as_dict(), whole_ix.hashes
    parts = [synth.build_index(full.shard(r, world)).as_dict() for r in range(world)]
    big = [int(t) for t in np.argsort(-whole_ix.sizes)[:7]]
    # the bitmap lists (>= 4096 postings on every shard: build_bitmaps' floor)
    assert all(len(parts[r][H[t]]) >= 4096 for r in range(world) for t in big[:5])
    rng = np.random.default_rng(11)
    cases = []
    for i in range(16):
        inc = [int(x) for x in rng.choice(big[:5], 3, replace=False)] + [int(rng.choice(big[5:]))]
        exc = [int(rng.choice([t for t in big if t not in inc]))] if i % 4 == 3 else []
        cases.append((inc, exc))
    c5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")

    def fn(r, ix):
        return ix.search_batch([Query([H[t] for t in inc], [H[t] for t in exc], now_ms=NOW, k=100,
                                      profile=(c5 if i % 2 else None)) for i, (inc, exc) in enumerate(cases)])

    res = _run_parts(parts, world, fn)
    for i, (inc, exc) in enumerate(cases):
        exp = orc.search(whole, [H[t] for t in inc], [H[t] for t in exc],
                         profile=(orc.profile_from(c5) if i % 2 else None), now_ms=NOW, k=100)
        for r in range(world):
            assert [(h.urlhash, h.score, h.tiebreak) for h in res[r][i]] == exp, (r, i)
