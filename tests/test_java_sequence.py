"""The Java drop-in's call sequence, replayed through the C ABI (ctypes).

java/net/yacy/kelondro/rwi/GpuTermSearch.java and
java/net/yacy/search/ranking/GpuReferenceOrder.java cannot be compiled here (no
JDK); this test makes exactly the libyrwi calls they make for one SearchEvent:

  TermSearch  -> GpuTermSearch(...): yrwi_list_size per include word (J1; no
                 CPU container is fetched), yrwi_join_exclude (joined rows)
  addRWIs     -> GpuReferenceOrder.normalizeWith -> yrwi_normalize_score on the
                 container's own rows: one settled score per row in a long[];
                 every queued entry carries its position, cardinal(e) =
                 scores[pos], fed in container order into rwiStack
                 (WeakPriorityBlockingQueue order)
  abstracts   -> GpuTermSearch.inclusion(): yrwi_get_list per include word (only
                 when asked); inclusionSizes() / abstracts(): yrwi_list_size,
                 yrwi_index_abstracts

and checks that the stack equals both the whole-query path (yrwi_query) and the
oracle (SearchEvent.java:697-816, ReferenceOrder.java:70,223), and that
inclusion() holds the index's lists (TermSearch.java:50-56)."""

import numpy as np
import pytest

import oracle as orc
from yacy_search_server_amd import RankingProfile, RWIIndex, synth

pytestmark = pytest.mark.gpu

NOW = 20741 * 86400000 + 4242


@pytest.fixture(scope="module")
def corpus():
    cfg = synth.preset("small")
    idx = synth.build_index(cfg)
    ix = RWIIndex(0)
    for t in range(cfg.n_terms):
        if idx.sizes[t]:
            ix.add(idx.hashes[t], idx.list_rows(t))
    yield cfg, idx, ix
    ix.close()


@pytest.mark.parametrize("profile", ["default", "c5", "date"])
def test_termsearch_then_reference_order(corpus, profile):
    cfg, idx, ix = corpus
    prof = {"default": RankingProfile(), "c5": RankingProfile("", "date=15,domlength=15,authority=13,tf=10"),
            "date": RankingProfile.date()}[profile]
    whole = idx.as_dict()
    n = 0
    for inc, exc in synth.queries(cfg, 24, 1, 3, 1, qseed=123):
        ih = [idx.hashes[t] for t in inc]
        eh = [idx.hashes[t] for t in exc]
        sizes = [ix.get_size(h) for h in ih]                          # GpuTermSearch: listSizes (J1)
        complete = all(sizes)
        rows = ix.term_search(ih, eh, now_ms=NOW)                     # GpuTermSearch: joinExclude
        assert np.array_equal(rows, orc.term_search(whole, ih, eh, 2147483647, NOW))
        if complete:                                                  # inclusion(), on demand: the lists
            for h in ih:
                assert np.array_equal(ix.get_list(h), whole[h])
        if len(rows) == 0:
            continue
        n += 1
        scores = ix.normalize_score(rows, prof, "en", NOW)            # GpuReferenceOrder.normalizeWith
        queue = list(range(len(rows)))                                # Entry(pos) per posting, container order
        ordered = np.array([scores[pos] for pos in queue], dtype=np.int64)  # cardinal(e) = scores[pos]
        stack = orc.topk(rows, ordered, 100)                          # rwiStack (WeakPriorityBlockingQueue)
        exp_scores, _ = orc.normalize_score(rows, orc.profile_from(prof), "en", NOW)
        assert np.array_equal(scores, exp_scores)
        assert stack == orc.search(whole, ih, eh, profile=orc.profile_from(prof), now_ms=NOW, k=100)
        got = ix.search(ih, eh, profile=prof, now_ms=NOW, k=100)    # the whole-query path
        assert [(h.urlhash, h.score, h.tiebreak) for h in got] == stack
    assert n > 0


def test_join_into_direct_buffer_and_query_stats(corpus):
    """GpuRWI.joinExcludeInto: the joined rows land in a caller-owned buffer of
    capacity/40 rows (JNI: a direct ByteBuffer); a buffer one row short is
    refused with YRWI_E_ARG.  GpuRWI.query(..., long[] stats): the call's
    yrwi_stats (joined rows = the container TermSearch returns)."""
    import ctypes
    from yacy_search_server_amd import _lib
    from yacy_search_server_amd._lib import CStats
    cfg, idx, ix = corpus
    lib = _lib.lib()
    done = 0
    for inc, exc in synth.queries(cfg, 12, 2, 3, 1, qseed=321):
        ih = b"".join(idx.hashes[t] for t in inc)
        eh = b"".join(idx.hashes[t] for t in exc)
        rows = ix.term_search([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], now_ms=NOW)
        m = len(rows)
        if m == 0:
            continue
        buf = np.zeros((m, 40), dtype=np.uint8)
        got = ctypes.c_int64()
        assert lib.yrwi_join_exclude(ix._h, ih, len(inc), eh, len(exc), 2147483647, NOW, buf.ctypes.data, m,
                                     ctypes.byref(got)) == 0
        assert got.value == m and np.array_equal(buf, rows)
        assert lib.yrwi_join_exclude(ix._h, ih, len(inc), eh, len(exc), 2147483647, NOW, buf.ctypes.data, m - 1,
                                     ctypes.byref(got)) == -1  # YRWI_E_ARG
        st = CStats()
        ix.search([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], now_ms=NOW, k=100, stats=st)
        assert st.postings_in == sum(int(idx.sizes[t]) for t in inc + exc)
        assert st.joined >= m and st.t_total_ns > 0
        done += 1
    assert done > 0


def test_inclusion_sizes_and_abstracts(corpus):
    """GpuTermSearch.inclusionSizes() / abstracts(): the IACount / IAResults that
    SearchEvent builds from inclusion() (SearchEvent.java:515-531), taken from the
    GPU index -- sizes equal the lists', each abstract equals the abstract of that
    word alone, and a query with an unknown word has neither (J1)."""
    cfg, idx, ix = corpus
    whole = idx.as_dict()
    done = 0
    for inc, _ in synth.queries(cfg, 8, 2, 3, 0, qseed=77):
        ih = [idx.hashes[t] for t in inc]
        sizes = [ix.get_size(h) for h in ih]
        assert sizes == [len(whole[h]) for h in ih]
        ab = ix.index_abstracts(ih)
        assert len(ab) == len(ih)
        for h, a in zip(ih, ab):
            assert ix.index_abstracts([h]) == [a] and a.startswith(b"{") and a.endswith(b"}")
        done += 1
    assert done > 0
    assert ix.index_abstracts([idx.hashes[inc[0]], b"AAAAAAAAAAAA"]) == []


def _jl_profile(name):
    import java_literal as jl
    if name == "default":
        return jl.RankingProfile()
    if name == "c5":
        return jl.RankingProfile.parse("", "date=15,domlength=15,authority=13,tf=10")
    p = jl.RankingProfile()
    p.all_zero()
    p.coeff_date = 15
    return p


@pytest.mark.parametrize("profile", ["default", "c5", "date"])
def test_reference_order_accumulates_across_arrivals(corpus, profile):
    """GpuReferenceOrder over one SearchEvent's arrivals (yrwi_event_order): the
    local container (RWIProcess.run, SearchEvent.java:631), a sitehost retry's
    container (:651), two remote peers' containers (Protocol.java:802; unsorted,
    duplicates inside and across) and a heuristic injection (Segment.java:758).
    One ReferenceOrder per SearchEvent: min/max, the max-distance fold and the host
    counts accumulate over every container (ReferenceOrder.java:163-216), and each
    container's postings are scored under the state after it -- equal, score for
    score, to the oracle's persistent ReferenceOrder (java_literal.ReferenceOrder).
    SearchEvent.addRWIs stays in Java: its doublecheck and rwiStack fed with those
    scores give the stack the GPU event path (yrwi_event_add) keeps; authority()
    reads the accumulated host counts."""
    import java_literal as jl
    cfg, idx, ix = corpus
    gp = {"default": RankingProfile(), "c5": RankingProfile("", "date=15,domlength=15,authority=13,tf=10"),
          "date": RankingProfile.date()}[profile]
    lp = _jl_profile(profile)
    whole = idx.as_dict()
    rng = np.random.default_rng({"default": 1, "c5": 2, "date": 3}[profile])
    qs = synth.queries(cfg, 6, 2, 3, 0, qseed=777)
    local = orc.term_search(whole, [idx.hashes[t] for t in qs[0][0]], [], 2147483647, NOW)
    retry = orc.term_search(whole, [idx.hashes[t] for t in qs[1][0]], [], 2147483647, NOW)
    allrows = np.asarray(idx.rows, dtype=np.uint8)
    remote = []
    for _ in range(3):
        take = rng.integers(0, len(allrows), 400)
        take[:80] = take[rng.integers(0, 400, 80)]  # duplicates inside the container
        r = allrows[take].copy()
        d = rng.random(400) < 0.5
        r[d, 38] = rng.integers(0, 40, int(d.sum()))  # word distances: the max-distance fold has work
        remote.append(r)
    arrivals = [(local, True), (retry, True), (remote[0], False), (remote[1], False), (remote[2], False)]
    total = sum(len(r) for r, _ in arrivals)
    order = jl.ReferenceOrder(lp, "en")
    stack = jl.ReverseQueue(3000)
    urls = set()
    # GpuReferenceOrder holds an order-only event (yrwi_event_open_order); the full
    # event beside it runs addRWIs on the GPU (yrwi_event_add) for comparison
    with ix.reference_order(gp, "en", NOW, max_hosts=total) as ev, \
            ix.event(gp, "en", NOW, k=3000, max_postings=total + 16) as ev_add:
        for rows, loc in arrivals:
            got = ev.order(rows, loc)                                   # GpuReferenceOrder.normalizeWith
            entries = order.normalize_with([bytes(x) for x in rows], NOW)
            assert got.tolist() == [order.cardinal(e) for e in entries]  # cardinal(e) of every posting
            for r, sc in zip(rows, got.tolist()):                       # SearchEvent.addRWIs (unchanged Java)
                h = bytes(r[:12])
                if h in urls:
                    continue
                urls.add(h)
                stack.put(sc, h)
            ev_add.add_rwis(rows, loc)
        hits, info = ev_add.results()
        assert [(h.urlhash, h.score) for h in hits] == [(h, w) for (w, _, h) in stack.items]
        hosts = sorted({bytes(r[6:12]) for r in allrows[rng.integers(0, len(allrows), 50)]})
        if lp.coeff_authority > 12:  # the host counts exist (and enter cardinal) only then
            assert ev.authority(hosts) == [order.authority(h) for h in hosts]
            assert info.maxdomcount == order.maxdomcount


def test_reference_order_events_reuse_memory_and_bound_hosts(corpus):
    """Order-only events (GpuReferenceOrder, one per SearchEvent) reuse closed
    events' device blocks: a second order after a first was closed starts from a
    clean state (the same scores as the first); an authority profile whose
    containers bring more hosts than max_hosts grows the event's host table
    (ReferenceOrder.doms is unbounded, ReferenceOrder.java:176-198): its scores
    and authority answers equal those of an event sized for all hosts."""
    cfg, idx, ix = corpus
    c5 = RankingProfile("", "date=15,domlength=15,authority=13,tf=10")
    rows = np.asarray(idx.rows, dtype=np.uint8)[:3000]
    firsts = []
    for _ in range(3):
        with ix.reference_order(c5, "en", NOW, max_hosts=4096) as ev:
            firsts.append(ev.order(rows[:1500], True).tolist())
            ev.order(rows[1500:], False)
    assert firsts[0] == firsts[1] == firsts[2]
    nhosts = len({bytes(r[6:12]) for r in rows})
    assert nhosts > 64
    hosts = sorted({bytes(r[6:12]) for r in rows})
    with ix.reference_order(c5, "en", NOW, max_hosts=4096) as big:
        want = [big.order(rows[a:b], a == 0).tolist() for a, b in ((0, 40), (40, 1000), (1000, 3000))]
        want_auth = big.authority(hosts)
    # max_hosts 8: 16 slots; the table grows at the second and third container
    for _ in range(2):  # the second round starts from a pooled (grown) block
        with ix.reference_order(c5, "en", NOW, max_hosts=8) as ev:
            got = [ev.order(rows[a:b], a == 0).tolist() for a, b in ((0, 40), (40, 1000), (1000, 3000))]
            assert got == want
            assert ev.authority(hosts) == want_auth


@pytest.mark.parametrize("kw", [dict(constraint=b"\0\0\x10\x01"), dict(language="de"), None])
def test_rwi_stack_pull_sources(corpus, kw):
    """GpuRWIStack (SearchEvent.addRWIs + pullOneRWI on the GPU): arrivals go to one
    filtered event (yrwi_event_add), hits come back in pullOneRWI(skipDoubleDom) order
    (yrwi_event_pull), and each pulled url's posting is found through
    yrwi_event_source -- the (arrival, row) the doublecheck admitted: the url's first
    posting that passed the constraints (SearchEvent.java:736-805), which may sit in a
    later arrival than the url's first posting.  Checked against the literal
    SearchEvent replayed arrival by arrival."""
    import java_literal as jl
    from yacy_search_server_amd import QueryFilter
    cfg, idx, ix = corpus
    rng = np.random.default_rng(21)
    allrows = np.asarray(idx.rows, dtype=np.uint8)
    arrivals = []
    for a in range(5):
        take = rng.integers(0, len(allrows), 500)
        take[:150] = take[rng.integers(0, 500, 150)]
        r = allrows[take].copy()
        r[rng.random(500) < 0.3, 29] ^= 0x10  # flag bits differ between postings of one url
        arrivals.append((r, a == 0))
    lf = jl.QueryFilter(**(kw or {}))
    ref = jl.SearchEventRWI(jl.RankingProfile(), "en", NOW, filt=lf)
    admitted = {}
    for a, (rows, loc) in enumerate(arrivals):
        ents = ref.order.normalize_with([bytes(x) for x in rows], NOW)
        for i, e in enumerate(ents):
            if ref.filt.admit(e):
                ref.q.put(ref.order.cardinal(e), e.urlHash)
                admitted.setdefault(e.urlHash, (a + 1, i))
    exp = ref.pull(300, True)
    gf = QueryFilter(**kw) if kw is not None else None
    with ix.event(RankingProfile(), "en", NOW, k=3000, filter=gf, max_postings=2600) as ev:
        for rows, loc in arrivals:
            ev.add_rwis(rows, loc)
        pulled = ev.pull(300, skip_double_dom=True)
        src = ev.source([h.urlhash for h in pulled])
        absent = ev.source([b"AAAAAAAAAAAA"])
    assert [(h.urlhash, h.score) for h in pulled] == exp
    assert absent == [(-1, -1)]
    for h, (a, i) in zip(pulled, src):
        assert (a, i) == admitted[h.urlhash]
        assert bytes(arrivals[a - 1][0][i][:12]) == h.urlhash
