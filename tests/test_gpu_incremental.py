"""Incremental url-dictionary maintenance (IndexCell.add keeps adding postings,
IndexCell.java:289): after the first full build, lists added, replaced and
removed are merged into the dictionary without re-sorting every key.  Every
step is checked three ways: the dictionary's own consistency (each posting's id
names its url hash, ids ascend in each list, the dictionary ascends), the query
results against the oracle on the current lists, and against a fresh index
built in full from the same lists (bit-exact hits)."""

import numpy as np
import pytest

import oracle as orc
from yacy_search_server_amd import Query, RankingProfile, RWIIndex, synth

pytestmark = pytest.mark.gpu

NOW = 20741 * 86400000 + 777


# every other query under an authority profile: its host counts key on the dense
# host ids the index records carry (ensure_host_ids), rebuilt after every change
C5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")


def _batch(qs, hashes):
    return [Query([hashes[t] for t in inc], [hashes[t] for t in exc], now_ms=NOW, k=50,
                  profile=(C5 if i % 2 else None)) for i, (inc, exc) in enumerate(qs)]


def _results(ix, lists, qs, hashes, fresh=None):
    batch = _batch(qs, hashes)
    got = [[(h.urlhash, h.score, h.tiebreak) for h in r] for r in ix.search_batch(batch)]
    if fresh is not None:
        assert got == fresh
    for qi, (inc, exc) in enumerate(qs):
        d = {hashes[t]: lists[hashes[t]] for t in inc + exc if hashes[t] in lists}
        prof = orc.profile_from(C5) if qi % 2 else None
        assert got[qi] == orc.search(d, batch[qi].include, batch[qi].exclude, profile=prof, now_ms=NOW, k=50), qi
    return got


def _fresh(lists, qs, hashes, monkeypatch):
    monkeypatch.setenv("YRWI_DICT_FULL", "1")
    ix = RWIIndex(0)
    try:
        for h, r in lists.items():
            ix.add(h, r)
        bad, nurls = ix.check_url_ids()
        assert bad == 0
        return [[(h.urlhash, h.score, h.tiebreak) for h in r] for r in ix.search_batch(_batch(qs, hashes))], nurls
    finally:
        ix.close()
        monkeypatch.delenv("YRWI_DICT_FULL")


def _mixed(a, b, rng):
    """rows of list a minus a third, plus rows of list b (new url hashes for a), unsorted"""
    keep = a[rng.random(len(a)) > 0.33]
    r = np.concatenate([keep, b[: max(1, len(b) // 2)]])
    return r[rng.permutation(len(r))]


_B64 = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
_RANK = bytes.maketrans(_B64, bytes(range(64)))


def _sorted_unique(rows):
    """RowSet order (Base64Order on the url hash), first occurrence of a url wins"""
    k = [bytes(r[:12]).translate(_RANK) for r in rows]
    o = sorted(range(len(rows)), key=lambda i: k[i])
    seen, out = set(), []
    for i in o:
        if k[i] not in seen:
            seen.add(k[i])
            out.append(rows[i])
    return np.array(out, dtype=np.uint8).reshape(-1, 40)


def test_incremental_dictionary(monkeypatch):
    cfg = synth.preset("tiny")
    idx = synth.build_index(cfg)
    hashes = idx.hashes
    rng = np.random.default_rng(7)
    terms = [t for t in range(len(hashes)) if idx.sizes[t]]
    rng.shuffle(terms)
    first, rest = terms[: len(terms) // 2], terms[len(terms) // 2:]
    qs = synth.queries(cfg, 40, 2, 3, 1)
    lists = {}
    ix = RWIIndex(0)
    try:
        for t in first:
            lists[hashes[t]] = idx.list_rows(t)
            ix.add(hashes[t], lists[hashes[t]])
        _results(ix, lists, qs, hashes)  # first query: full build
        bad, n0 = ix.check_url_ids()
        assert bad == 0
        steps = []
        # 1: new lists, mostly new url hashes
        steps.append([("add", t, idx.list_rows(t)) for t in rest[: len(rest) // 3]])
        # 2: a list whose urls are all in the dictionary already (no id moves)
        donor = lists[hashes[first[0]]]
        steps.append([("add", terms[-1], donor[::2].copy())])
        # 3: replaced lists (a third dropped, another list's rows mixed in) and a removal
        steps.append([("put", first[1], _mixed(lists[hashes[first[1]]], idx.list_rows(rest[-2]), rng)),
                      ("put", first[2], _mixed(lists[hashes[first[2]]], idx.list_rows(rest[-3]), rng)),
                      ("del", first[3], None)])
        # 4: the remaining lists
        steps.append([("add", t, idx.list_rows(t)) for t in rest[len(rest) // 3:-1]])
        nprev = n0
        base = ix.index_info()
        assert base["full_rebuilds"] == 1 and base["incremental_updates"] == 0, base
        for si, step in enumerate(steps):
            for op, t, rows in step:
                h = hashes[t]
                if op == "del":
                    ix.add(h, np.zeros((0, 40), dtype=np.uint8))
                    lists.pop(h, None)
                elif op == "put":
                    ix.add(h, rows, sorted=False)
                    lists[h] = _sorted_unique(rows)
                else:
                    ix.add(h, rows)
                    lists[h] = rows
            before = ix.index_info()
            bad, nurls = ix.check_url_ids()
            assert bad == 0, si
            after = ix.index_info()
            if si in (1, 2):  # small changes: merged into the dictionary, not rebuilt
                assert after["incremental_updates"] == before["incremental_updates"] + 1, (si, after)
                assert after["full_rebuilds"] == before["full_rebuilds"], (si, after)
            assert nurls >= nprev, si  # keys of removed postings stay until a full rebuild
            if si == 1:
                assert nurls == nprev  # no new key: nothing moved
            nprev = nurls
            exp, nfull = _fresh(lists, qs, hashes, monkeypatch)
            assert nfull <= nurls
            _results(ix, lists, qs, hashes, fresh=exp)
    finally:
        ix.close()


def test_incremental_with_bitmap_lists(monkeypatch):
    """A bitmap-sized list (>= 1/64 of the url ids) replaced incrementally: the
    remapped ids, line heads and bitmaps must give the oracle's results."""
    cfg = synth.preset("small")
    idx = synth.build_index(cfg)
    hashes = idx.hashes
    rng = np.random.default_rng(11)
    lists = {hashes[t]: idx.list_rows(t) for t in range(len(hashes)) if idx.sizes[t]}
    big = [int(t) for t in np.argsort(-idx.sizes)[:4]]
    qs = [([big[0], big[1]], []), ([big[1], big[2]], [big[3]]), ([big[0], big[3], big[2]], [])]
    qs += synth.queries(cfg, 30, 2, 3, 1)
    ix = RWIIndex(0)
    try:
        for h, r in lists.items():
            ix.add(h, r)
        _results(ix, lists, qs, hashes)
        info = ix.index_info()
        assert info["bitmap_lists"] > 0, info
        # the largest list loses a third of its rows and gains rows of another list (new urls for it)
        h = hashes[big[0]]
        new = _mixed(lists[h], idx.list_rows(big[5] if len(big) > 5 else int(np.argsort(-idx.sizes)[5])), rng)
        ix.add(h, new, sorted=False)
        lists[h] = _sorted_unique(new)
        bad, _ = ix.check_url_ids()
        assert bad == 0
        info2 = ix.index_info()
        assert info2["incremental_updates"] == info["incremental_updates"] + 1, info2
        assert info2["bitmap_lists"] > 0, info2
        exp, _ = _fresh(lists, qs, hashes, monkeypatch)
        _results(ix, lists, qs, hashes, fresh=exp)
    finally:
        ix.close()


def test_index_memory_repacked(monkeypatch):
    """A list re-put again and again (IndexCell.add): the replaced lists' device
    memory is reclaimed (index arena repacked once dead bytes pass the live ones),
    so the arena stays bounded, and the results stay exact across the moves."""
    monkeypatch.setenv("YRWI_REPACK_MIN_MB", "1")
    cfg = synth.preset("small")
    idx = synth.build_index(cfg)
    hashes = idx.hashes
    rng = np.random.default_rng(3)
    top = [int(t) for t in np.argsort(-idx.sizes)[:40]]  # a small live index: the re-puts dominate the arena
    lists = {hashes[t]: idx.list_rows(t) for t in top}
    big = top[:6]
    qs = [([big[0], big[1]], []), ([big[0], big[2]], [big[3]])]
    qs += [([int(a), int(b)], []) for a, b in rng.choice(top, size=(18, 2), replace=True) if a != b]
    ix = RWIIndex(0)
    try:
        for h, r in lists.items():
            ix.add(h, r)
        _results(ix, lists, qs, hashes)
        first = ix.index_info()
        h = hashes[big[0]]
        for it in range(24):
            donor = idx.list_rows(big[1 + it % 5])
            new = _mixed(lists[h], donor, rng)
            ix.add(h, new, sorted=False)
            lists[h] = _sorted_unique(new)
            if it % 6 == 5:
                _results(ix, lists, qs, hashes)
        bad, _ = ix.check_url_ids()
        assert bad == 0
        last = ix.index_info()
        assert last["repacks"] > 0, last
        # reclaimed: at most the live lists plus the dead bytes that trigger the next repack
        # (the live bytes again); without repacks the 24 re-puts alone add ~2x the live index
        live = sum(len(r) for r in lists.values()) * 85
        assert last["index_bytes_used"] < 2.2 * live + (16 << 20), (last, live)
        _results(ix, lists, qs, hashes)
    finally:
        ix.close()
