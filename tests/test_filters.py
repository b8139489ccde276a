"""addRWIs constraints and the doubledom pull order.

CPU: the literal oracle (oracle/java_literal.py QueryFilter / pull_double_dom)
against hand-derived expectations of SearchEvent.java:736-806 (filters),
:2459-2474 (testFlags) and :1297-1394 (pullOneRWI).
GPU: libyrwi (filter predicates fused into k_score, k_doubledom) against the
literal oracle on seeded corpora, mixed filtered / unfiltered batches.
No reference test covers these paths (parity pinned by the restatement)."""

import numpy as np
import pytest

import java_literal as jl
from yacy_search_server_amd import synth

NOW = 20741 * 86400000


def _row(h, flags=b"\0\0\0\0", doctype=b"t", lang=b"en", pos=1):
    return jl.make_row(h, 30, 3, 2, 1, 100, 10, pos, 1, 100, NOW - 86400000 * 30, NOW, lang, doctype[0], 0, 0, 0,
                       flags)


def _bits(*js):
    b = bytearray(4)
    for j in js:
        b[j >> 3] |= 1 << (j & 7)
    return bytes(b)


def _vars(row):
    return jl.Vars.from_row(row, NOW)


def test_testflags_any_all():
    f_any = jl.QueryFilter(constraint=_bits(3, 20))
    f_all = jl.QueryFilter(constraint=_bits(3, 20), all_of_constraint=True)
    r1, r2, r3 = _row(b"AAAAAAhostAA", _bits(20)), _row(b"BBBBBBhostAA", _bits(3, 20, 7)), _row(b"CCCCCChostAA")
    assert [f_any.admit(_vars(r)) for r in (r1, r2, r3)] == [True, True, False]
    assert [f_all.admit(_vars(r)) for r in (r1, r2, r3)] == [False, True, False]


def test_contentdom_strict_and_flags():
    img_flag = _row(b"AAAAAAhostAA", _bits(20), b"t")
    img_type = _row(b"BBBBBBhostAA", _bits(), b"i")
    app = _row(b"CCCCCChostAA", _bits(23), b"t")
    f = jl.QueryFilter(contentdom=1)
    fs = jl.QueryFilter(contentdom=1, strict_contentdom=True)
    fa = jl.QueryFilter(contentdom=4, strict_contentdom=True)
    assert [f.admit(_vars(r)) for r in (img_flag, img_type, app)] == [True, False, False]
    assert [fs.admit(_vars(r)) for r in (img_flag, img_type, app)] == [False, True, False]
    assert [fa.admit(_vars(r)) for r in (img_flag, img_type, app)] == [False, False, True]  # APP: flag even if strict
    assert jl.QueryFilter(contentdom=0).admit(_vars(img_type))  # TEXT (code 0) does not filter


def test_language_site_doublecheck_flagcount():
    de = _row(b"AAAAAAhostAA", _bits(0, 31), lang=b"de")
    en = _row(b"BBBBBBhostBB", _bits(0))
    assert [jl.QueryFilter(language="de").admit(_vars(r)) for r in (de, en)] == [True, False]
    assert not jl.QueryFilter(language="deu").admit(_vars(de))
    f = jl.QueryFilter(sitehash=b"hostBB")
    assert [f.admit(_vars(r)) for r in (de, en)] == [False, True]
    f = jl.QueryFilter(sitehash=b"hostXX", alt_sitehash=b"hostAA")
    assert [f.admit(_vars(r)) for r in (de, en)] == [True, False]
    f = jl.QueryFilter(siteexcludes=[b"hostAA"])
    assert [f.admit(_vars(r)) for r in (de, en)] == [False, True]
    f = jl.QueryFilter(urlhashes=[b"AAAAAAhostAA"], language="xx")
    assert [f.admit(_vars(r)) for r in (de, en)] == [False, False]
    # the doublechecked row is not counted, the language-dropped one is
    assert f.flagcount[0] == 1 and f.flagcount[31] == 0


def test_pull_double_dom_order():
    def st(hosts):
        return [(b"%06d" % i + h.encode() * 6, 100 - i) for i, h in enumerate(hosts)]
    s = st("AABACB")
    got = [x[0][6] for x in jl.pull_double_dom(s, 6)]
    assert bytes(got) == b"ABCAAB"
    # 10 polls per round: after ten doubles one queued entry is emitted first
    s = st("A" * 12 + "B")
    got = bytes(x[0][6] for x in jl.pull_double_dom(s, 13))
    assert got == b"AAB" + b"A" * 10
    assert len(jl.pull_double_dom(s, 5)) == 5 and jl.pull_double_dom([], 5) == []


# ------------------------------------------------------------------- GPU
def _corpus(preset, seed=3):
    cfg = synth.preset(preset)
    idx = synth.build_index(cfg)
    rng = np.random.default_rng(seed)
    rows = idx.rows
    rows[:, 21] = rng.choice(np.frombuffer(b"tiam", np.uint8), len(rows))  # doctypes for strict contentdom
    return cfg, idx


def _filters(idx, rng):
    hosts = sorted({bytes(r[6:12]) for r in idx.rows[rng.integers(0, len(idx.rows), 200)]})
    urls = [bytes(r[:12]) for r in idx.rows[rng.integers(0, len(idx.rows), 300)]]
    return [
        ("any", dict(constraint=_bits(20, 24))),
        ("all", dict(constraint=_bits(24, 25), all_of_constraint=True)),
        ("image", dict(contentdom=1)),
        ("audio_strict", dict(contentdom=2, strict_contentdom=True)),
        ("app", dict(contentdom=4)),
        ("lang_de", dict(language="de")),
        ("site", dict(sitehash=hosts[0], alt_sitehash=hosts[1])),
        ("siteex", dict(siteexcludes=hosts[:50])),
        ("doublecheck", dict(urlhashes=urls)),
        ("doubledom", dict(skip_double_dom=True)),
        ("doubledom_lang", dict(skip_double_dom=True, language="en", siteexcludes=hosts[:20])),
    ]


@pytest.mark.gpu
@pytest.mark.parametrize("preset", ["dense", "tiny"])
def test_filters_gpu_match_literal(preset):
    from yacy_search_server_amd import Query, QueryFilter, RWIIndex
    cfg, idx = _corpus(preset)
    rng = np.random.default_rng(11)
    lit_index = {h: [bytes(r) for r in rows] for h, rows in idx.as_dict().items()}
    ix = RWIIndex(0)
    try:
        for h, rows in idx.as_dict().items():
            ix.add(h, rows)
        qs = synth.queries(cfg, 6, 1, 2, 1, qseed=21)
        big = [int(t) for t in np.argsort(-idx.sizes)[:3]]
        qs = [q for p in zip(qs, [([big[0]], []), ([big[1]], [big[2]]), ([big[0], big[2]], [])] * 2) for q in p]
        fl = _filters(idx, rng)
        batch, exp = [], []
        for n, (name, kw) in enumerate(fl * 2):
            inc, exc = qs[n % len(qs)]
            incl = [idx.hashes[t] for t in inc]
            excl = [idx.hashes[t] for t in exc]
            k = [10, 100, 37][n % 3]
            gf = QueryFilter(**kw)
            lf = jl.QueryFilter(**kw)
            batch.append(Query(incl, excl, k=k, now_ms=NOW, filter=gf))
            e = jl.search(lit_index, incl, excl, jl.RankingProfile(), "en", now_ms=NOW, k=k, filt=lf)
            exp.append((name, e, lf.flagcount))
            batch.append(Query(incl, excl, k=k, now_ms=NOW))  # unfiltered neighbour in the same batch
            exp.append((name + "/none", jl.search(lit_index, incl, excl, jl.RankingProfile(), "en", now_ms=NOW, k=k),
                        None))
        got = ix.search_batch(batch)
        changed = 0
        for i, (q, g, (name, e, fc)) in enumerate(zip(batch, got, exp)):
            assert [(h.urlhash, h.score) for h in g] == e, name
            if fc is not None:
                assert q.filter.flagcount == fc, name
                changed += e != exp[i + 1][1]
        assert changed >= len(fl)  # the filters did change most results
    finally:
        ix.close()


@pytest.mark.gpu
def test_doubledom_gpu_few_hosts():
    """Eight hosts only, so pullOneRWI's host rotation and its 10-poll rounds decide the order."""
    import heap
    from yacy_search_server_amd import QueryFilter, RWIIndex
    cfg, idx = _corpus("dense")
    hosts = [b"hst%03d" % i for i in range(8)]
    d = {}
    for h, rows in idx.as_dict().items():
        r = rows.copy()
        sel = np.frombuffer(b"".join(hosts), np.uint8).reshape(8, 6)
        r[:, 6:12] = sel[r[:, 3] % 8]  # host from a url-hash char: deterministic, uneven
        d[h] = heap.sort_unique(r)
    lit = {h: [bytes(x) for x in rows] for h, rows in d.items()}
    ix = RWIIndex(0)
    try:
        for h, rows in d.items():
            ix.add(h, rows)
        big = [h for h, _ in sorted(d.items(), key=lambda kv: -len(kv[1]))[:3]]
        for inc in ([big[0]], [big[1], big[2]]):
            for k in (10, 100, 3000):
                f = QueryFilter(skip_double_dom=True)
                g = ix.search(inc, [], now_ms=NOW, k=k, filter=f)
                e = jl.search(lit, inc, [], jl.RankingProfile(), "en", now_ms=NOW, k=k,
                              filt=jl.QueryFilter(skip_double_dom=True))
                assert [(x.urlhash, x.score) for x in g] == e, (len(inc), k)
                plain = jl.search(lit, inc, [], jl.RankingProfile(), "en", now_ms=NOW, k=k)
                if k <= 100 and len(e) > 8:
                    assert e != plain
    finally:
        ix.close()
