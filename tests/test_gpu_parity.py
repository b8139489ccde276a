"""GPU parity (MI355X): libyrwi's HIP path vs the oracle, bit-exact.

Every check goes through the C ABI (yacy_search_server_amd.rwi -> libyrwi.so).
Sizes are ones the C++ oracle finishes in seconds."""

import numpy as np
import pytest

import java_literal as jl
import oracle as orc
from kat_util import kat_index, kat_profile, load_kats, run_kat
from yacy_search_server_amd import Query, RankingProfile, RWIIndex, synth

pytestmark = pytest.mark.gpu

NOW = 20741 * 86400000 + 4242
KATS = [k for k in load_kats() if "lists" in k]


def _rp(jlprof):
    rp = RankingProfile()
    for _, f in jl.PROFILE_FIELDS:
        setattr(rp, f, getattr(jlprof, f))
    return rp


class GpuEngine:
    def _ix(self, idx):
        ix = RWIIndex(0)
        for h, rows in idx.items():
            ix.add(h, rows)
        return ix

    def term_search(self, idx, incl, excl, md, now):
        ix = self._ix(idx)
        try:
            return ix.term_search(incl, excl, md, now)
        finally:
            ix.close()

    def search(self, idx, incl, excl, prof, lang, md, now, k):
        ix = self._ix(idx)
        try:
            return [(h.urlhash, h.score) for h in ix.search(incl, excl, _rp(prof), lang, md, now, k)]
        finally:
            ix.close()


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_kat_gpu(kat):
    run_kat(GpuEngine(), kat)


@pytest.fixture(scope="module", params=["dense", "tiny", "small"])
def corpus(request):
    cfg = synth.preset(request.param)
    idx = synth.build_index(cfg)
    ix = RWIIndex(0)
    for t in range(cfg.n_terms):
        if idx.sizes[t]:
            ix.add(idx.hashes[t], idx.list_rows(t))
    yield cfg, idx, ix
    ix.close()


def _profiles():
    c5 = jl.RankingProfile.parse("", "date=15,domlength=15,authority=13,tf=10")
    date = jl.RankingProfile()
    date.all_zero()
    date.coeff_date = 15
    rng = np.random.default_rng(3)
    rnd = jl.RankingProfile()
    for _, f in jl.PROFILE_FIELDS:
        setattr(rnd, f, int(rng.integers(0, 16)))
    rnd.coeff_urlcomps = 27
    return [("default", jl.RankingProfile()), ("c5", c5), ("date", date), ("rand", rnd)]


def test_join_rows_bit_exact(corpus):
    cfg, idx, ix = corpus
    d = idx.as_dict()
    for i, (inc, exc) in enumerate(synth.queries(cfg, 25, 1, 4, 1, qseed=11)):
        ih = [idx.hashes[t] for t in inc]
        eh = [idx.hashes[t] for t in exc]
        for md in (2147483647, 60):
            for now in (NOW, 15500 * 86400000 + 7):
                exp = orc.term_search(d, ih, eh, md, now)
                got = ix.term_search(ih, eh, md, now)
                assert got.shape == exp.shape and np.array_equal(got, exp), (i, md, now)


def test_topk_bit_exact(corpus):
    cfg, idx, ix = corpus
    d = idx.as_dict()
    qs = synth.queries(cfg, 20, 1, 4, 1, qseed=12)
    for pname, prof in _profiles():
        for now in (NOW, 15500 * 86400000 + 7):
            batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], k=100,
                           profile=_rp(prof), now_ms=now) for inc, exc in qs]
            got = ix.search_batch(batch)
            for qi, (q, g) in enumerate(zip(batch, got)):
                exp = orc.search(d, q.include, q.exclude, orc.profile_from(prof), "en", now_ms=now, k=100)
                assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp, (pname, now, qi)


def test_normalize_score_bit_exact(corpus):
    cfg, idx, ix = corpus
    d = idx.as_dict()
    for inc, exc in synth.queries(cfg, 8, 1, 3, 0, qseed=13):
        ih = [idx.hashes[t] for t in inc]
        rows = orc.term_search(d, ih, [], 2147483647, NOW)
        if len(rows) == 0:
            continue
        for pname, prof in _profiles():
            exp, _ = orc.normalize_score(rows, orc.profile_from(prof), "en", NOW)
            got = ix.normalize_score(rows, _rp(prof), "en", NOW)
            assert np.array_equal(got, exp), pname


def test_batch_equals_single_and_k_edges(corpus):
    cfg, idx, ix = corpus
    qs = synth.queries(cfg, 10, 1, 3, 1, qseed=14)
    batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], k=k, now_ms=NOW)
             for (inc, exc), k in zip(qs, [1, 5, 100, 3000, 0, 77, 2048, 2049, 10, 100])]
    got = ix.search_batch(batch)
    for q, g in zip(batch, got):
        single = ix.search(q.include, q.exclude, k=q.k, now_ms=NOW)
        assert [(h.urlhash, h.score) for h in g] == [(h.urlhash, h.score) for h in single]
        assert len(g) <= q.k
    d = idx.as_dict()
    for q, g in zip(batch, got):
        exp = orc.search(d, q.include, q.exclude, now_ms=NOW, k=q.k) if q.k else []
        assert [(h.urlhash, h.score) for h in g] == [(h, s) for h, s, _ in exp]


def test_missing_and_duplicate_terms(corpus):
    cfg, idx, ix = corpus
    d = idx.as_dict()
    a, b = idx.hashes[0], idx.hashes[1]
    missing = b"ZZZZZZZZZZZZ"
    for inc, exc in [([a, missing], []), ([a], [missing]), ([a, a], []), ([a, b, a], [b]), ([], [a])]:
        got = [(h.urlhash, h.score) for h in ix.search(inc, exc, now_ms=NOW)]
        exp = [(h, s) for h, s, _ in orc.search(d, inc, exc, now_ms=NOW)]
        assert got == exp


def test_fold_overflow_paths():
    """Adversarial posintext order (strictly increasing) forces the chunk- and
    shard-level fold summaries to overflow; the exact fallbacks must agree."""
    rng = np.random.default_rng(5)
    for n in (3000, 9000):
        rows = np.zeros((n, 40), dtype=np.uint8)
        alpha = np.frombuffer(jl.ALPHA, dtype=np.uint8)
        for i in range(n):
            h = jl.key_to_hash((i + 1) << 20 | 7)
            rows[i, :12] = np.frombuffer(h, dtype=np.uint8)
        rows[:, 12:14] = np.frombuffer((15000).to_bytes(2, "big"), dtype=np.uint8)
        rows[:, 17] = 0
        rows[:, 18] = 50
        rows[:, 21] = ord("t")
        rows[:, 22:24] = np.frombuffer(b"en", dtype=np.uint8)
        p = np.arange(1, n + 1) if n == 3000 else np.maximum.accumulate(rng.integers(1, 60000, n))
        rows[:, 34] = (p >> 8) & 0xFF
        rows[:, 35] = p & 0xFF
        rows[:, 38] = rng.integers(0, 256, n)
        rows[:, 33] = rng.integers(1, 20, n)
        ix = RWIIndex(0)
        for name, prof in _profiles():
            exp, nm = orc.normalize_score(rows, orc.profile_from(prof), "en", NOW)
            got = ix.normalize_score(rows, _rp(prof), "en", NOW)
            assert np.array_equal(got, exp), name
        ix.add(b"TERMover____", rows)
        got = [(h.urlhash, h.score) for h in ix.search([b"TERMover____"], now_ms=NOW, k=200)]
        exp = [(h, s) for h, s, _ in orc.search({b"TERMover____": rows}, [b"TERMover____"], now_ms=NOW, k=200)]
        assert got == exp
        ix.close()


def test_fold_many_record_chunks():
    """Containers of 100+ chunks whose posintext trends upwards with noise: record
    chunks (new prefix max) sit between runs of non-record chunks in every batch of
    64 chunk summaries k_shard_fin folds, some chunks have posintext 0 throughout."""
    rng = np.random.default_rng(11)
    for n, step in ((300000, 40), (260000, 400)):
        rows = np.zeros((n, 40), dtype=np.uint8)
        alpha = np.frombuffer(jl.ALPHA, dtype=np.uint8)
        keys = np.arange(1, n + 1, dtype=np.int64) * 977 + 13
        for j in range(12):
            rows[:, 11 - j] = alpha[(keys >> (6 * j)) & 63]
        rows[:, 12:14] = np.frombuffer((15000).to_bytes(2, "big"), dtype=np.uint8)
        rows[:, 18] = 50
        rows[:, 21] = ord("t")
        rows[:, 22:24] = np.frombuffer(b"en", dtype=np.uint8)
        p = np.minimum(65535, np.arange(n) // step + rng.integers(0, 2500, n))
        p[(np.arange(n) // 2048) % 7 == 3] = 0
        rows[:, 34] = (p >> 8) & 0xFF
        rows[:, 35] = p & 0xFF
        rows[:, 38] = rng.integers(0, 256, n) * (rng.random(n) < 0.3)
        rows[:, 33] = rng.integers(1, 20, n)
        ix = RWIIndex(0)
        ix.add(b"TERMmany____", rows)
        got = [(h.urlhash, h.score) for h in ix.search([b"TERMmany____"], now_ms=NOW, k=100)]
        exp = [(h, s) for h, s, _ in orc.search({b"TERMmany____": rows}, [b"TERMmany____"], now_ms=NOW, k=100)]
        assert got == exp
        ix.close()


def test_put_list_validation():
    ix = RWIIndex(0)
    good = synth.build_index(synth.preset("dense")).list_rows(0)
    bad = good.copy()
    bad[3, 0] = ord("!")
    with pytest.raises(Exception):
        ix.add(b"TERMbad_____", bad)
    unsorted = good[::-1].copy()
    with pytest.raises(Exception):
        ix.add(b"TERMuns_____", unsorted, sorted=True)
    ix.add(b"TERMuns_____", unsorted, sorted=False)
    assert ix.get_size(b"TERMuns_____") == len(good)
    # Index.get: the stored list comes back sorted, byte for byte (yrwi_get_list)
    assert np.array_equal(ix.get_list(b"TERMuns_____"), good)
    assert ix.get_list(b"TERMnone____").shape == (0, 40)
    nolang = good.copy()
    nolang[0, 22:24] = 0
    with pytest.raises(Exception):
        ix.add(b"TERMnol_____", nolang)
    ix.close()


@pytest.mark.slow
def test_c1_sample_bit_exact():
    """C1 (1M URLs x 10k words, 10M postings): 40 queries, full top-100."""
    cfg = synth.preset("C1")
    qs = synth.queries(cfg, 40, 2, 3, 1, qseed=21)
    need = sorted({t for inc, exc in qs for t in inc + exc})
    idx = synth.build_index(cfg, terms=np.array(need))
    ix = RWIIndex(0)
    for t in need:
        if idx.sizes[t]:
            ix.add(idx.hashes[t], idx.list_rows(t))
    d = idx.as_dict()
    batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], now_ms=NOW) for inc, exc in qs]
    got = ix.search_batch(batch)
    for q, g in zip(batch, got):
        exp = orc.search(d, q.include, q.exclude, now_ms=NOW, k=100)
        assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp
    ix.close()


@pytest.fixture(scope="module")
def long_lists():
    """C2's eight longest lists (0.7-3.7 M postings each, every one with a url-id
    bitmap), resident on one context."""
    cfg = synth.preset("C2")
    df = synth.counts(cfg)
    big = [int(t) for t in np.argsort(-df, kind="stable")[:8]]
    idx = synth.build_index(cfg, terms=np.array(sorted(big)))
    ix = RWIIndex(0)
    for t in big:
        ix.add(idx.hashes[t], idx.list_rows(t))
    yield cfg, df, big, idx, ix
    ix.close()


@pytest.mark.parametrize("band_order", ["1", "0"])
def test_long_bitmap_tiles_and_schedules(long_lists, band_order, monkeypatch):
    """3-4 term queries with an excluded term over lists of >= 2^18 postings: the
    deferred fold steps and the exclusion probe take 2048-id bitmap tiles
    (k_probe<true>, BM_LARGE_MIN), the final step 1024-id tiles; in band-major
    order (default) and in job order (YRWI_BAND_ORDER=0) the results are the
    oracle's, byte for byte (the schedules only reorder tiles)."""
    monkeypatch.setenv("YRWI_BAND_ORDER", band_order)
    cfg, df, big, idx, ix = long_lists
    assert df[big[-1]] >= (1 << 18)
    rng = np.random.default_rng(5)
    qs = []
    for _ in range(12):
        pick = [int(x) for x in rng.permutation(big)[:5]]
        n = int(rng.integers(3, 5))
        qs.append((pick[:n], pick[n:n + 1]))
    d = idx.as_dict()
    batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], now_ms=NOW) for inc, exc in qs]
    got = ix.search_batch(batch)
    for q, g in zip(batch, got):
        exp = orc.search(d, q.include, q.exclude, now_ms=NOW, k=100)
        assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp


@pytest.mark.parametrize("j5", [("1", None), ("0", None), ("1", "0.06")], ids=["j5", "no_j5", "j5_largest_only"])
def test_j5_side_arrays(long_lists, j5, monkeypatch):
    """The joined side's J5 words come from the 16-B side arrays of the bitmap
    lists (DList::j5), from the 32-B records (YRWI_J5=0), or from either when
    YRWI_J5_GB leaves only the largest list one: enumeration steps, the deferred
    folds of 3-4 term queries and the final top-k equal the oracle's."""
    monkeypatch.setenv("YRWI_J5", j5[0])
    if j5[1]:
        monkeypatch.setenv("YRWI_J5_GB", j5[1])
    cfg, df, big, idx, _ = long_lists
    ix = RWIIndex(0)
    try:
        for t in big:
            ix.add(idx.hashes[t], idx.list_rows(t))
        d = idx.as_dict()
        rng = np.random.default_rng(8)
        for n in (2, 2, 3, 4):
            pick = [int(x) for x in rng.permutation(big)[:n]]
            ih = [idx.hashes[t] for t in pick]
            for md in (2147483647, 60):
                assert np.array_equal(ix.term_search(ih, [], md, NOW), orc.term_search(d, ih, [], md, NOW)), (pick, md)
        batch = [Query([idx.hashes[t] for t in rng.permutation(big)[:int(rng.integers(2, 5))]], [], now_ms=NOW)
                 for _ in range(8)]
        for q, g in zip(batch, ix.search_batch(batch)):
            assert [(h.urlhash, h.score, h.tiebreak) for h in g] == orc.search(d, q.include, q.exclude, now_ms=NOW, k=100)
    finally:
        ix.close()


@pytest.mark.parametrize("chain", ["1", "0"], ids=["chained", "stepwise"])
def test_dense_bitmap_joins(long_lists, chain, monkeypatch):
    """Joins of dense bitmap lists (the bitmap probe; round 5 also enumerated the
    AND of both bitmaps here, removed in round 6): term_search rows, top-k with
    tie-breaks, with and without excluded terms and a distance filter, stepwise
    (YRWI_NO_CHAIN=1: every fold step a join job) and chained."""
    monkeypatch.setenv("YRWI_NO_CHAIN", "1" if chain == "0" else "0")
    cfg, df, big, idx, ix = long_lists
    d = idx.as_dict()
    rng = np.random.default_rng(13)
    for n in (2, 2, 3):
        pick = [int(x) for x in rng.permutation(big)[:n + 1]]
        ih = [idx.hashes[t] for t in pick[:n]]
        for eh, md in (([], 2147483647), ([idx.hashes[pick[n]]], 2147483647), ([], 60)):
            assert np.array_equal(ix.term_search(ih, eh, md, NOW), orc.term_search(d, ih, eh, md, NOW)), (pick, md)
    batch = []
    for i in range(12):
        pick = [int(x) for x in rng.permutation(big)]
        ni, ne = 2 + i % 3, (i // 3) % 2
        batch.append(Query([idx.hashes[t] for t in pick[:ni]], [idx.hashes[t] for t in pick[ni:ni + ne]], now_ms=NOW))
    for q, g in zip(batch, ix.search_batch(batch)):
        assert [(h.urlhash, h.score, h.tiebreak) for h in g] == orc.search(d, q.include, q.exclude, now_ms=NOW, k=100)


@pytest.mark.parametrize("ratio", ["1", "1000000000"])
def test_forced_join_algorithm(corpus, ratio, monkeypatch):
    """Every join/exclusion step through the probe kernel (ratio 1) or through
    merge-path tiles (huge ratio): results identical to the oracle either way."""
    monkeypatch.setenv("YRWI_PROBE_RATIO", ratio)
    cfg, idx, ix = corpus
    d = idx.as_dict()
    for inc, exc in synth.queries(cfg, 12, 1, 4, 1, qseed=31):
        ih = [idx.hashes[t] for t in inc]
        eh = [idx.hashes[t] for t in exc]
        assert np.array_equal(ix.term_search(ih, eh, 2147483647, NOW), orc.term_search(d, ih, eh, 2147483647, NOW))
        got = [(h.urlhash, h.score) for h in ix.search(ih, eh, now_ms=NOW)]
        assert got == [(h, s) for h, s, _ in orc.search(d, ih, eh, now_ms=NOW)]


def _keyed_rows(keys, seed):
    """Valid 40-B rows whose url hashes are jl.key_to_hash(key) (ascending keys -> sorted list)."""
    rng = np.random.default_rng(seed)
    n = len(keys)
    rows = np.zeros((n, 40), dtype=np.uint8)
    for i, k in enumerate(keys):
        rows[i, :12] = np.frombuffer(jl.key_to_hash(int(k) << 20 | 7), dtype=np.uint8)
    rows[:, 12:14] = np.frombuffer((15000).to_bytes(2, "big"), dtype=np.uint8)
    rows[:, 18] = 50
    rows[:, 21] = ord("t")
    rows[:, 22:24] = np.frombuffer(b"en", dtype=np.uint8)
    p = rng.integers(1, 3000, n)
    rows[:, 34] = (p >> 8) & 0xFF
    rows[:, 35] = p & 0xFF
    rows[:, 33] = rng.integers(1, 20, n)
    rows[:, 38] = rng.integers(0, 40, n)
    return rows


@pytest.mark.parametrize("chain", ["1", "0"], ids=["chained", "stepwise"])
@pytest.mark.parametrize("algo", ["probe", "merge"])
def test_compaction_pieces(algo, chain, monkeypatch):
    """The normalisation pieces the compaction writes (k_compact_sum, one per tile)
    in place of k_reduce's chunk summaries: 2- and 3-term joins whose posintext
    rises along the url order (a tile's records overflow its SEGC segments and
    k_shard_fin rewalks the tile's run), runs of posintext 0, empty tiles; probe
    and merge tiles, chained and stepwise folds; profiles without authority beside
    queries with exclusions or authority (k_reduce's path) in one batch."""
    monkeypatch.setenv("YRWI_PROBE_RATIO", "1" if algo == "probe" else "1000000000")
    monkeypatch.setenv("YRWI_NO_CHAIN", "1" if chain == "0" else "0")
    rng = np.random.default_rng(17)
    n = 20000
    keys = np.arange(n)

    def rows_for(sel, seed, mode):
        r = _keyed_rows(keys[sel], seed)
        m = len(r)
        if mode == "rise":
            p = np.minimum(65535, np.arange(1, m + 1) * 3)
        elif mode == "noisy":
            p = np.minimum(65535, np.arange(m) // 8 + rng.integers(0, 200, m))
            p[(np.arange(m) // 300) % 5 == 2] = 0
        else:
            p = rng.integers(0, 3000, m)
        r[:, 34] = (p >> 8) & 0xFF
        r[:, 35] = p & 0xFF
        r[:, 38] = rng.integers(0, 256, m) * (rng.random(m) < 0.5)
        return r

    d = {
        b"TERMpcA_____": rows_for(np.ones(n, bool), 1, "rise"),
        b"TERMpcB_____": rows_for(rng.random(n) < 0.6, 2, "noisy"),
        b"TERMpcC_____": rows_for(rng.random(n) < 0.3, 3, "rand"),
        b"TERMpcD_____": rows_for(rng.random(n) < 0.05, 4, "rise"),
        b"TERMpcE_____": rows_for(rng.random(n) < 0.5, 5, "rand"),
    }
    A, B, C, D, E = list(d)
    ix = RWIIndex(0)
    try:
        for h, r in d.items():
            ix.add(h, r)
        qs = [([A, B], []), ([B, A], []), ([A, C], []), ([B, D], []), ([A, B, C], []), ([A, C, D], []),
              ([A, B], [E]), ([A, B, C], [E]), ([D, E], [])]
        for pname, prof in _profiles():
            batch = [Query(inc, exc, k=100, profile=_rp(prof), now_ms=NOW) for inc, exc in qs]
            for qi, (q, g) in enumerate(zip(batch, ix.search_batch(batch))):
                exp = orc.search(d, q.include, q.exclude, orc.profile_from(prof), "en", now_ms=NOW, k=100)
                assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp, (pname, qi)
    finally:
        ix.close()


@pytest.mark.parametrize("nab", [(2048, 2048), (2047, 2050), (4095, 4097), (6000, 6289), (12288, 1)])
def test_merge_tile_boundaries(nab, monkeypatch):
    """Merge-path tiles (forced) over lists whose combined length sits on and
    around multiples of the tile size, every B key matching: matches on both
    sides of each tile split and the lookahead element must all be joined once."""
    monkeypatch.setenv("YRWI_PROBE_RATIO", "1000000000")
    na, nb = nab
    a = _keyed_rows(np.arange(na), 1)
    b = _keyed_rows(np.arange(0, 2 * nb, 2)[:nb], 2)
    d = {b"TERMtileA___": a, b"TERMtileB___": b}
    ix = RWIIndex(0)
    try:
        for h, r in d.items():
            ix.add(h, r)
        q = [b"TERMtileA___", b"TERMtileB___"]
        for md in (2147483647, 100):
            assert np.array_equal(ix.term_search(q, [], md, NOW), orc.term_search(d, q, [], md, NOW)), md
            assert np.array_equal(ix.term_search(q[:1], q[1:], md, NOW), orc.term_search(d, q[:1], q[1:], md, NOW))
        got = [(h.urlhash, h.score) for h in ix.search(q, now_ms=NOW, k=300)]
        assert got == [(h, s) for h, s, _ in orc.search(d, q, now_ms=NOW, k=300)]
    finally:
        ix.close()


@pytest.mark.parametrize("mode", ["probe", "count_first"])
def test_bitmap_unit_boundaries(mode, monkeypatch):
    """Url-id bitmaps in 16-B units of 96 ids (yrwi_bitmap.h): lists whose ids sit
    on both sides of every unit's word boundaries (ids 96v + 0/31/32/63/64/95),
    the first and the last url id, a url space that is not a multiple of 96.  A
    (every id) and C (every third) and B (the boundary ids) have bitmaps, D (ids
    96v + 95 and 96v + 96, below the bitmap minimum) has none: 2-4 term joins,
    an exclusion, through the bitmap probe and the count-first popcounts
    (YRWI_CHAIN_CF=2) -- rows and top-k equal to the oracle's."""
    monkeypatch.setenv("YRWI_CHAIN_CF", "2" if mode == "count_first" else "1")
    m = 96 * 1000 + 37
    keys = np.arange(m)
    r = keys % 96
    sel_b = np.isin(r, (0, 31, 32, 63, 64, 95)) | (keys == 0) | (keys == m - 1)
    d = {b"TERMunitA___": _keyed_rows(keys, 11), b"TERMunitB___": _keyed_rows(keys[sel_b], 12),
         b"TERMunitC___": _keyed_rows(keys[keys % 3 == 0], 13),
         b"TERMunitD___": _keyed_rows(keys[(r == 95) | ((r == 0) & (keys > 0))][:3000], 14)}
    A, B, C, D = d
    ix = RWIIndex(0)
    try:
        for h, rows in d.items():
            ix.add(h, rows)
        for inc, exc in (([A, B], []), ([B, C], []), ([A, B, C], []), ([A, C, B, D], []), ([B, C], [D]),
                         ([A, B, C], [D]), ([C, A], [B])):
            assert np.array_equal(ix.term_search(inc, exc, 2147483647, NOW),
                                  orc.term_search(d, inc, exc, 2147483647, NOW)), (inc, exc)
            got = [(h.urlhash, h.score) for h in ix.search(inc, exc, now_ms=NOW, k=200)]
            assert got == [(h, s) for h, s, _ in orc.search(d, inc, exc, now_ms=NOW, k=200)], (inc, exc)
    finally:
        ix.close()


@pytest.mark.parametrize("gb", ["0.000001", "0.002"])
def test_batch_split_by_scratch_budget(corpus, gb, monkeypatch):
    """A batch larger than the scratch budget runs as consecutive passes over
    query ranges (one query per pass at the tiny budget): same hits as the oracle,
    each query's hits at its own position."""
    monkeypatch.setenv("YRWI_SCRATCH_GB", gb)
    cfg, idx, ix = corpus
    d = idx.as_dict()
    qs = synth.queries(cfg, 24, 1, 4, 1, qseed=41)
    batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], k=k, now_ms=NOW)
             for (inc, exc), k in zip(qs, [100, 7, 3000, 1] * 6)]
    got = ix.search_batch(batch)
    for qi, (q, g) in enumerate(zip(batch, got)):
        exp = orc.search(d, q.include, q.exclude, now_ms=NOW, k=q.k)
        assert [(h.urlhash, h.score) for h in g] == [(h, s) for h, s, _ in exp], (gb, qi)


def _collision_family(base, n_blocks=6):
    """64 url hashes with one Java hashCode: 6 two-char blocks, each either
    (x, y) or (x + 1, y - 31) -- equal 31 * x + y."""
    out = []
    for m in range(1 << n_blocks):
        h = bytearray(base[:12 - 2 * n_blocks])
        for j in range(n_blocks):
            x, y = base[12 - 2 * n_blocks + 2 * j], base[12 - 2 * n_blocks + 2 * j + 1]
            h += bytes([x + 1, y - 31]) if (m >> j) & 1 else bytes([x, y])
        out.append(bytes(h))
    return out


def test_treeset_dedupe_across_chunks():
    """Many postings tying in (score, ByteArray.hashCode) spread over several
    2048-posting chunks: the TreeSet keeps the first arrival of each class, so
    chunk lists lose entries to the dedupe and the per-query top-k must go on
    below its first selection.  k from 10 to 3000."""
    rng = np.random.default_rng(17)
    fam = []
    for f in range(120):
        # x in A..Y, y in g..x: (x + 1, y - 31) is again a pair of valid url-hash characters
        base = bytes(rng.choice(np.frombuffer(jl.ALPHA[:26], dtype=np.uint8), 2)) + b"".join(
            bytes([int(rng.integers(65, 90)), int(rng.integers(97 + 6, 97 + 25))]) for _ in range(5))
        fam.append((f, _collision_family(base, 5)))
    hashes = {}
    for f, hs in fam:
        assert len({jl.bytearray_hashcode(h) for h in hs}) == 1
        for h in hs:
            hashes.setdefault(h, f)
    filler = set()
    while len(filler) < 5000:
        h = bytes(rng.choice(np.frombuffer(jl.ALPHA, dtype=np.uint8), 12))
        if h not in hashes:
            filler.add(h)
    allh = sorted(list(hashes) + list(filler), key=jl.key72)
    n = len(allh)
    rows = np.zeros((n, 40), dtype=np.uint8)
    for i, h in enumerate(allh):
        rows[i, :12] = np.frombuffer(h, dtype=np.uint8)
        f = hashes.get(h)
        day = 20000 + f if f is not None else 15000 + int(rng.integers(0, 300))  # families rank first
        rows[i, 12:14] = np.frombuffer(day.to_bytes(2, "big"), dtype=np.uint8)
        rows[i, 17:19] = np.frombuffer((40 + (f or 0) % 7).to_bytes(2, "big"), dtype=np.uint8)
        rows[i, 21] = ord("t")
        rows[i, 22:24] = np.frombuffer(b"en", dtype=np.uint8)
        rows[i, 33] = 9 if f is not None else int(rng.integers(1, 9))
        p = 3 if f is not None else int(rng.integers(1, 400))
        rows[i, 34], rows[i, 35] = p >> 8, p & 0xFF
    term = b"TERMdedupe__"
    ix = RWIIndex(0)
    ix.add(term, rows)
    d = {term: rows}
    for k in (10, 100, 1000, 3000):
        got = [(h.urlhash, h.score, h.tiebreak) for h in ix.search([term], now_ms=NOW, k=k)]
        exp = orc.search(d, [term], [], now_ms=NOW, k=k)
        assert got == exp, k
    ix.close()


def _cqueries(batch):
    from yacy_search_server_amd._lib import CQuery
    import ctypes
    arr = (CQuery * len(batch))()
    keep = []
    for i, q in enumerate(batch):
        ib = ctypes.create_string_buffer(b"".join(q.include), max(1, 12 * len(q.include)))
        eb = ctypes.create_string_buffer(b"".join(q.exclude), max(1, 12 * len(q.exclude)))
        prof = RankingProfile()
        keep += [ib, eb, prof]
        arr[i].incl = ctypes.cast(ib, ctypes.c_void_p)
        arr[i].nincl = len(q.include)
        arr[i].excl = ctypes.cast(eb, ctypes.c_void_p)
        arr[i].nexcl = len(q.exclude)
        arr[i].max_distance = q.max_distance
        arr[i].k = q.k
        arr[i].profile = ctypes.pointer(prof.c)
        arr[i].language = b"en"
        arr[i].now_ms = q.now_ms
    return arr, keep


def test_async_batches_pinned_and_pageable(corpus):
    """yrwi_query_batch_submit/_wait: several batches in flight on the lanes, results
    in pinned (yrwi_host_alloc, written by the GPU directly) and in pageable buffers,
    equal to the synchronous batch call and to the oracle."""
    import ctypes
    from yacy_search_server_amd._lib import CHit, CStats
    cfg, idx, ix = corpus
    d = idx.as_dict()
    batches = []
    for s in range(4):
        qs = synth.queries(cfg, 9 + s, 1, 3, s % 2, qseed=40 + s)
        batches.append([Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], k=50, now_ms=NOW)
                        for inc, exc in qs])
    kmax = 50
    tickets = []
    for s, b in enumerate(batches):
        arr, keep = _cqueries(b)
        if s % 2:
            hits, nout = ix.host_array(CHit, len(b) * kmax), ix.host_array(ctypes.c_int32, len(b))
        else:
            hits, nout = (CHit * (len(b) * kmax))(), (ctypes.c_int32 * len(b))()
        st = CStats()
        tickets.append((ix.submit_raw(arr, len(b), kmax, hits, nout, st), b, hits, nout, st, keep, arr))
    for t, b, hits, nout, st, keep, arr in tickets:
        ix.wait(t)
        assert st.postings_in > 0
        sync = ix.search_batch(b, kmax=kmax)
        for i, q in enumerate(b):
            got = [(bytes(hits[i * kmax + j].urlhash), hits[i * kmax + j].score) for j in range(nout[i])]
            assert got == [(h.urlhash, h.score) for h in sync[i]]
            exp = orc.search(d, q.include, q.exclude, now_ms=NOW, k=q.k)
            assert got == [(h, s) for h, s, _ in exp]
    with pytest.raises(Exception):
        ix.wait(tickets[0][0])  # a ticket is collected once


def test_stats_compact_accounting(corpus):
    """yrwi_stats: a two-term query joins in one step, so k_compact's algorithmic
    bytes are the joined rows times 96 (enumeration: 12 B pair + url id, 32 B
    record of the accumulated side, 16 B of the joined side, 36 B written) or 80
    (by test: one 32-B record gathered), and its HIP-event time is positive
    whenever rows were joined."""
    from yacy_search_server_amd._lib import CStats
    cfg, idx, ix = corpus
    seen = 0
    for inc, _ in synth.queries(cfg, 12, 2, 2, 0, qseed=77):
        if len(set(inc)) < 2:
            continue
        st = CStats()
        ix.search_batch([Query([idx.hashes[t] for t in inc], [], k=20, now_ms=NOW)], stats=st)
        if st.joined == 0:
            continue
        seen += 1
        assert st.bytes_compact in (96 * st.joined, 80 * st.joined), (st.bytes_compact, st.joined)
        assert st.t_compact_ns > 0
    assert seen > 0


def test_null_stats_production_path(corpus):
    """The production call passes no yrwi_stats (NULL: no HIP events around the
    kernel groups) -- the path bench.py times and a JNI caller runs.  Batches of
    mixed shapes, eight in flight on the lanes through yrwi_query_batch_submit
    with st == NULL, and synchronous yrwi_query_batch calls with st == NULL:
    every result equals the oracle's."""
    import ctypes
    from yacy_search_server_amd._lib import CHit
    cfg, idx, ix = corpus
    d = idx.as_dict()
    kmax = 100
    pend = []
    for s in range(10):
        qs = synth.queries(cfg, 6 + s, 1 + s % 3, 2 + s % 3, s % 2, qseed=900 + s)
        b = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], k=kmax, now_ms=NOW) for inc, exc in qs]
        arr, keep = _cqueries(b)
        hits, nout = ix.host_array(CHit, len(b) * kmax), ix.host_array(ctypes.c_int32, len(b))
        pend.append((ix.submit_raw(arr, len(b), kmax, hits, nout, None), b, hits, nout, keep, arr))
    for t, b, hits, nout, keep, arr in pend:
        ix.wait(t)
        for i, q in enumerate(b):
            got = [(bytes(hits[i * kmax + j].urlhash), hits[i * kmax + j].score) for j in range(nout[i])]
            exp = orc.search(d, q.include, q.exclude, now_ms=NOW, k=q.k)
            assert got == [(h, s) for h, s, _ in exp]
    # synchronous, NULL statistics
    t, b, _, _, keep, arr = pend[3]
    hits, nout = (CHit * (len(b) * kmax))(), (ctypes.c_int32 * len(b))()
    ix.search_batch_raw(arr, len(b), kmax, hits, nout, None)
    for i, q in enumerate(b):
        got = [(bytes(hits[i * kmax + j].urlhash), hits[i * kmax + j].score) for j in range(nout[i])]
        assert got == [(h, s) for h, s, _ in orc.search(d, q.include, q.exclude, now_ms=NOW, k=q.k)]


@pytest.mark.parametrize("chain", ["1", "0", "cf"], ids=["chained", "stepwise", "count_first"])
def test_chained_folds_corpus(corpus, chain, monkeypatch):
    """Chained folds (ChainQ: one join step, then k_chain tests each match against
    the later include lists and the exclusion lists) and the step-by-step fold
    (YRWI_NO_CHAIN=1): 2-4 include terms with 0-2 excluded terms, plus quoted
    queries (maxDistance: never chained); results equal the oracle's, tie-breaks
    included.  count_first (YRWI_CHAIN_CF=2): every 3- and 4-term chained fold counts
    list 0 x list 1 apart and chains its survivors from list 2 (ChainQ::perm) --
    in the benchmarks only folds whose list 2 is the smallest, which these small
    lists (no int-wrapped J2 keys) never produce."""
    monkeypatch.setenv("YRWI_NO_CHAIN", "1" if chain == "0" else "0")
    monkeypatch.setenv("YRWI_CHAIN_CF", "2" if chain == "cf" else "1")
    cfg, idx, ix = corpus
    d = idx.as_dict()
    qs = synth.queries(cfg, 40, 2, 4, 2, qseed=2024) + synth.queries(cfg, 20, 3, 4, 0, qseed=2025)
    batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], now_ms=NOW,
                   max_distance=(len(inc) - 1 if i % 7 == 3 else 2147483647)) for i, (inc, exc) in enumerate(qs)]
    got = ix.search_batch(batch)
    for q, g in zip(batch, got):
        exp = orc.search(d, q.include, q.exclude, max_distance=q.max_distance, now_ms=NOW, k=100)
        assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp
    for q in batch[:10]:
        assert np.array_equal(ix.term_search(q.include, q.exclude, q.max_distance, NOW),
                              orc.term_search(d, q.include, q.exclude, q.max_distance, NOW))


@pytest.mark.parametrize("bm,cf", [("64", "1"), ("0", "1"), ("64", "2"), ("0", "2")],
                         ids=["bitmaps", "no_bitmaps", "bitmaps_count_first", "no_bitmaps_count_first"])
def test_chained_folds_long_lists(long_lists, bm, cf, monkeypatch):
    """Chained folds over C2's eight longest lists: with url-id bitmaps every later
    list is tested by one bitmap word per match; without (YRWI_BM_DIV=0) by the
    list's ids staged around the tile's range in LDS, or -- ranges longer than the
    LDS stage -- through the line heads (k_chain_part / k_chain)."""
    monkeypatch.setenv("YRWI_BM_DIV", bm)
    monkeypatch.setenv("YRWI_CHAIN_CF", cf)
    cfg, df, big, idx, _ = long_lists
    ix = RWIIndex(0)
    try:
        for t in big:
            ix.add(idx.hashes[t], idx.list_rows(t))
        d = idx.as_dict()
        rng = np.random.default_rng(11)
        batch = []
        for i in range(16):
            pick = [int(x) for x in rng.permutation(big)]
            ni = 2 + i % 3
            ne = (i // 3) % 3
            batch.append(Query([idx.hashes[t] for t in pick[:ni]], [idx.hashes[t] for t in pick[ni:ni + ne]],
                               now_ms=NOW))
        for q, g in zip(batch, ix.search_batch(batch)):
            assert [(h.urlhash, h.score, h.tiebreak) for h in g] == orc.search(d, q.include, q.exclude, now_ms=NOW,
                                                                               k=100)
    finally:
        ix.close()


def _restrict(d, sel):
    """ReferenceContainerCache.get(key, urlselection) (ReferenceContainerCache.java:448-470) for
    every list: the rows whose url hash is in the selection, in their order; an emptied list is
    what searchConjunction treats as absent (AbstractIndex.java:118-121)."""
    s = set(sel)
    out = {}
    for h, rows in d.items():
        r = rows[np.fromiter((bytes(x[:12]) in s for x in rows), dtype=bool, count=len(rows))]
        if len(r):
            out[h] = r
    return out


def test_urlselection_restricts_every_list(corpus):
    """TermSearch's urlselection (yrwi_query_desc.urlselection): every include and exclude
    list restricted to the selected urls before the conjunction, so J1, the J2 fold order and
    every J3 dispatch see the restricted sizes -- single lists (rows as stored), chained folds
    of 2-4 terms with exclusions; selections small and large, with urls the index does not
    hold.  Equal to the oracle over the restricted lists; a quoted (maxDistance) fold with a
    selection is refused."""
    from yacy_search_server_amd._lib import YrwiError
    cfg, idx, ix = corpus
    d = idx.as_dict()
    urls = np.unique(np.asarray(idx.rows)[:, :12].copy().view("S12").ravel())
    rng = np.random.default_rng(606)
    qs = synth.queries(cfg, 24, 1, 4, 2, qseed=808)
    for trial, frac in enumerate((0.002, 0.05, 0.4)):
        m = max(1, int(frac * len(urls)))
        sel = [bytes(u) for u in rng.choice(urls, m, replace=False)]
        sel += [b"AAAAAAAAAAA" + bytes([65 + i]) for i in range(3)]  # not in the index
        rd = _restrict(d, sel)
        batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], now_ms=NOW, urlselection=sel)
                 for inc, exc in qs]
        for q, g in zip(batch, ix.search_batch(batch)):
            exp = orc.search(rd, q.include, q.exclude, now_ms=NOW, k=100)
            assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp, trial
        for q in batch[:8]:
            assert np.array_equal(ix.term_search(q.include, q.exclude, 2147483647, NOW, urlselection=sel),
                                  orc.term_search(rd, q.include, q.exclude, 2147483647, NOW)), trial
    two = next((inc for inc, _ in qs if len(set(inc)) >= 2), None)
    if two is not None:
        with pytest.raises(YrwiError):
            ix.search_batch([Query([idx.hashes[t] for t in two], [], max_distance=1, now_ms=NOW, urlselection=sel)])


@pytest.mark.parametrize("maxb", [None, "4", "1"])
def test_authority_host_partition(corpus, maxb, monkeypatch):
    """Authority (coeff_authority > 12) host counts by partition: every query's
    hosts hashed into buckets (k_hpart_hist / k_hpart_scatter), each bucket
    counted in LDS (k_hbucket), every element's count written for cardinal and the
    largest folded into maxdomcount.  YRWI_HPART_MAXB caps the buckets per query:
    at 1 a query over the biggest lists has thousands of hosts in its one bucket,
    which overflow the LDS table into the query's global host table.  Bit-exact
    against the oracle (ReferenceOrder.java:176-216, 223-265)."""
    if maxb:
        monkeypatch.setenv("YRWI_HPART_MAXB", maxb)
    cfg, idx, ix = corpus
    d = idx.as_dict()
    big = [int(t) for t in np.argsort(-idx.sizes)[:4]]
    qs = [([big[0]], []), ([big[1]], []), ([big[0], big[1]], []), ([big[0]], [big[2]])]
    qs += synth.queries(cfg, 12, 1, 3, 1, qseed=44)
    c5 = jl.RankingProfile.parse("", "date=15,domlength=15,authority=13,tf=10")
    a14 = jl.RankingProfile()
    a14.coeff_authority = 14
    for prof in (c5, a14):
        batch = [Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], k=100, profile=_rp(prof),
                       now_ms=NOW) for inc, exc in qs]
        got = ix.search_batch(batch)
        for qi, (q, g) in enumerate(zip(batch, got)):
            exp = orc.search(d, q.include, q.exclude, orc.profile_from(prof), "en", now_ms=NOW, k=100)
            assert [(h.urlhash, h.score, h.tiebreak) for h in g] == exp, (maxb, qi)
