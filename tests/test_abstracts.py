"""Index abstracts and the secondary-search join.

Serving side: WordReferenceFactory.compressIndex (WordReferenceFactory.java:
75-117) per include word (htroot/yacy/search.java:264-281).  Asking side:
decompressIndex (:125-155), SecondarySearchSuperviser.addAbstract (:43-65),
SetTools.joinConstructive (:76-116) and prepareSecondarySearch (:117-196).

CPU: the restatement (oracle/abstracts.py) against hand-derived values.
GPU: yrwi_index_abstracts and yrwi_secondary_search against the restatement,
byte-exact, on synthetic lists and abstracts from several peers."""

import numpy as np
import pytest

import abstracts as ab
from yacy_search_server_amd import synth

ALPHA = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"


def _row(url: bytes) -> bytes:
    return url + bytes(28)


def test_compress_index_hand():
    c = [_row(b"AAAAAAhost01"), _row(b"BBBBBBhost01"), _row(b"CCCCCChost00"), _row(b"DDDDDD-ost02")]
    assert ab.compress_index(c) == b"{-ost02:DDDDDD,host00:CCCCCC,host01:AAAAAABBBBBB}"
    assert ab.compress_index(c, exclude=[_row(b"BBBBBBhost01")]) == b"{-ost02:DDDDDD,host00:CCCCCC,host01:AAAAAA}"
    assert ab.compress_index([]) == b"{}"


def test_decompress_index_hand():
    t = b"{-ost02:DDDDDD,host00:CCCCCC,host01:AAAAAABBBBBB}"
    m = ab.decompress_index(t, b"peerAAAAAAAA")
    assert m == {u: {b"peerAAAAAAAA"} for u in (b"DDDDDD-ost02", b"CCCCCChost00", b"AAAAAAhost01", b"BBBBBBhost01")}
    assert ab.decompress_index(b"-ost02:DDDDDD", b"p" * 12) == {}        # no braces: empty map
    assert ab.decompress_index(b"{}", b"p" * 12) == {}
    assert ab.decompress_index(b"{host00:CCCCCC,garbage}", b"p" * 12) == {b"CCCCCChost00": {b"p" * 12}}
    with pytest.raises(ValueError):
        ab.decompress_index(b"{host00:CCCCCCC}", b"p" * 12)
    assert ab.decompress_index(b"{host00:CCCCC}", b"p" * 12) == {}  # shorter than 13: the loop never runs


def test_add_abstract_keeps_newest_peer():
    s = ab.SecondarySearch()
    s.add_abstract(b"w" * 12, {b"u1": {b"p1"}, b"u2": {b"p1"}})
    s.add_abstract(b"w" * 12, {b"u1": {b"p2"}})
    assert s.cache[b"w" * 12] == {b"u1": {b"p2"}, b"u2": {b"p1"}}


def test_join_and_plan_hand():
    s = ab.SecondarySearch()
    w1, w2 = b"W1__________", b"W2__________"
    s.add_abstract(w1, {b"u1": {b"pA"}, b"u2": {b"pB"}, b"u3": {b"pA"}})
    s.add_abstract(w2, {b"u1": {b"pB"}, b"u3": {b"pA"}})
    join, plan = s.prepare([w1, w2], mypeer=b"pZ")
    # w2 is smaller (2 * 1000 + 1 < 3 * 1000 + 0): its peer sets are kept
    assert join == {b"u1": {b"pB"}, b"u3": {b"pA"}}
    assert plan == [(b"pA", [b"u3"], [w1, w2]), (b"pB", [b"u1"], [w2])]
    # asked peers are not asked again
    assert s.prepare([w1, w2], mypeer=b"pZ")[1] == []


def _urls(rng, n, nhosts):
    hosts = [bytes(ALPHA[int(x)] for x in rng.integers(0, 64, 6)) for _ in range(nhosts)]
    out = set()
    while len(out) < n:
        out.add(bytes(ALPHA[int(x)] for x in rng.integers(0, 64, 6)) + hosts[int(rng.integers(0, nhosts))])
    return sorted(out)


@pytest.mark.gpu
def test_index_abstracts_gpu():
    from yacy_search_server_amd import RWIIndex
    cfg = synth.preset("tiny")
    idx = synth.build_index(cfg)
    order = [int(t) for t in np.argsort(-idx.sizes)[:5]]
    ix = RWIIndex(0)
    try:
        for t in range(cfg.n_terms):
            if idx.sizes[t]:
                ix.add(idx.hashes[t], idx.list_rows(t))
        terms = [idx.hashes[t] for t in order]
        got = ix.index_abstracts(terms)
        exp = [ab.compress_index([bytes(r) for r in idx.list_rows(t)]) for t in order]
        assert got == exp
        got = ix.index_abstracts(terms[:2], exclude=terms[2])
        ex = [bytes(r) for r in idx.list_rows(order[2])]
        assert got == [ab.compress_index([bytes(r) for r in idx.list_rows(t)], ex) for t in order[:2]]
        assert ix.index_abstracts(terms[:2] + [b"ZZZZZZZZZZZZ"]) == []
        # hosts with many urls: one list built from few hosts
        rng = np.random.default_rng(4)
        rows = np.zeros((5000, 40), dtype=np.uint8)
        b64 = sorted(_urls(rng, 5000, 7), key=lambda u: [ALPHA.index(c) for c in u])  # Base64Order
        for i, u in enumerate(b64):
            rows[i, :12] = np.frombuffer(u, dtype=np.uint8)
        rows[:, 22:24] = ord("e")
        ix.add(b"fewhostsAAAA", rows)
        assert ix.index_abstracts([b"fewhostsAAAA"]) == [ab.compress_index([bytes(r) for r in rows])]
    finally:
        ix.close()


def _peer_abstracts(rng, words, npeers, base):
    """every peer holds a random part of each word's url universe; arrival order shuffled"""
    peers = sorted({bytes(ALPHA[int(x)] for x in rng.integers(0, 64, 12)) for _ in range(npeers)})
    out = []
    for p in peers:
        for w in words:
            sel = [u for u in base[w] if rng.random() < 0.4]
            out.append((w, p, ab.compress_index([_row(u) for u in sel])))
    order = rng.permutation(len(out))
    return [out[i] for i in order], peers


def _oracle_plan(abstracts, words, mypeer, checked=()):
    s = ab.SecondarySearch()
    s.checked = set(checked)
    for w, p, t in abstracts:
        s.add_abstract(w, ab.decompress_index(t, p))
    return s.prepare(words, mypeer)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_secondary_search_gpu(seed):
    from yacy_search_server_amd import RWIIndex
    rng = np.random.default_rng(seed)
    words = sorted(bytes(ALPHA[int(x)] for x in rng.integers(0, 64, 12)) for _ in range(3))
    common = _urls(rng, 3000, 40)
    base = {w: sorted(set(common[: 2000]) | set(_urls(rng, 1500, 30))) for w in words}
    abstracts, peers = _peer_abstracts(rng, words, 9, base)
    ix = RWIIndex(0)
    try:
        for mypeer, checked in ((peers[0], ()), (b"notapeer____", peers[1:3])):
            join, wl, plan = ix.secondary_search(abstracts, len(words), mypeer, checked)
            ejoin, eplan = _oracle_plan(abstracts, words, mypeer, checked)
            assert wl == words
            assert join == [(u, next(iter(ejoin[u]))) for u in sorted(ejoin)]
            assert plan == eplan
        # not every word has abstracts yet: nothing planned
        assert ix.secondary_search(abstracts, len(words) + 1, peers[0])[2] == []
        # a text without braces contributes nothing; a malformed one is refused
        extra = abstracts + [(words[0], peers[1], b"xx:AAAAAA")]
        join, _, plan = ix.secondary_search(extra, len(words), peers[0])
        ejoin, eplan = _oracle_plan(extra, words, peers[0])
        assert plan == eplan and len(join) == len(ejoin)
        from yacy_search_server_amd._lib import YrwiError
        with pytest.raises(YrwiError):
            ix.secondary_search(abstracts + [(words[0], peers[1], b"{host00:AAAAAAA}")], len(words), peers[0])
    finally:
        ix.close()
