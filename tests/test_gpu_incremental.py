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
from yacy_search_server_amd import Query, RWIIndex, synth

pytestmark = pytest.mark.gpu

NOW = 20741 * 86400000 + 777


def _results(ix, lists, qs, hashes, fresh=None):
    batch = [Query([hashes[t] for t in inc], [hashes[t] for t in exc], now_ms=NOW, k=50) for inc, exc in qs]
    got = [[(h.urlhash, h.score, h.tiebreak) for h in r] for r in ix.search_batch(batch)]
    if fresh is not None:
        assert got == fresh
    for qi, (inc, exc) in enumerate(qs):
        d = {hashes[t]: lists[hashes[t]] for t in inc + exc if hashes[t] in lists}
        assert got[qi] == orc.search(d, batch[qi].include, batch[qi].exclude, now_ms=NOW, k=50), qi
    return got


def _fresh(lists, qs, hashes, monkeypatch):
    monkeypatch.setenv("YRWI_DICT_FULL", "1")
    ix = RWIIndex(0)
    try:
        for h, r in lists.items():
            ix.add(h, r)
        bad, nurls = ix.check_url_ids()
        assert bad == 0
        batch = [Query([hashes[t] for t in inc], [hashes[t] for t in exc], now_ms=NOW, k=50) for inc, exc in qs]
        return [[(h.urlhash, h.score, h.tiebreak) for h in r] for r in ix.search_batch(batch)], nurls
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
            bad, nurls = ix.check_url_ids()
            assert bad == 0, si
            assert nurls >= nprev, si  # keys of removed postings stay until a full rebuild
            if si == 1:
                assert nurls == nprev  # no new key: nothing moved
            nprev = nurls
            exp, nfull = _fresh(lists, qs, hashes, monkeypatch)
            assert nfull <= nurls
            _results(ix, lists, qs, hashes, fresh=exp)
    finally:
        ix.close()
