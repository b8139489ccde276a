"""Oracle pinning (CPU): both restatements against the reference's known-answer
tests and the per-quirk KATs of tests/golden/kats.json, and against each other
on seeded random indexes."""

import numpy as np
import pytest

import java_literal as jl
import oracle as orc
from kat_util import load_kats, run_kat
from yacy_search_server_amd import synth

KATS = load_kats()
ROW_KATS = [k for k in KATS if "lists" in k]


class LiteralEngine:
    def term_search(self, idx, incl, excl, md, now):
        d = {h: [bytes(r) for r in rows] for h, rows in idx.items()}
        rows = jl.term_search(d, incl, excl, md, now)
        return np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(-1, 40)

    def search(self, idx, incl, excl, prof, lang, md, now, k):
        d = {h: [bytes(r) for r in rows] for h, rows in idx.items()}
        return jl.search(d, incl, excl, prof, lang, md, now, k)


class CppEngine:
    def term_search(self, idx, incl, excl, md, now):
        return orc.term_search(idx, incl, excl, md, now)

    def search(self, idx, incl, excl, prof, lang, md, now, k):
        return [(h, s) for h, s, _ in orc.search(idx, incl, excl, orc.profile_from(prof), lang, md, now, k)]


@pytest.mark.parametrize("kat", ROW_KATS, ids=[k["name"] for k in ROW_KATS])
@pytest.mark.parametrize("engine", [LiteralEngine(), CppEngine()], ids=["literal", "cpp"])
def test_kat(engine, kat):
    run_kat(engine, kat)


def test_kat_distance_fold_state():
    kat = next(k for k in KATS if k["name"] == "n3_distance_fold_negative_term")
    from kat_util import kat_index, kat_profile
    idx = kat_index(kat)
    rows = idx[b"TERMfold____"]
    _, nm = orc.normalize_score(rows, orc.profile_from(kat_profile(kat)), "en", kat["now_ms"])
    assert nm.max_distance_D == kat["expect_norm"]["D"]
    order = jl.ReferenceOrder(kat_profile(kat), "en")
    order.normalize_with([bytes(r) for r in rows], kat["now_ms"])
    assert order.max.distance() == 40 and order.min.distance() == 0


def test_wordreferencevarstest_min():
    """WordReferenceVarsTest.testMin (WordReferenceVarsTest.java:40-95), on the literal Vars."""
    now = 20000 * jl.DAY
    h = b"kN0WkdoVHAAA"
    r5 = jl.make_row(h, 20, 3, 2, 1, 1, 1, 5, 1, 100, now, now, b"en", ord("t"), 0, 0, 0, b"\0\0\0\0")
    r30 = jl.make_row(h, 20, 3, 2, 1, 1, 1, 30, 1, 100, now, now, b"en", ord("t"), 0, 0, 0, b"\0\0\0\0")
    wv_min = jl.Vars.from_row(r5, now)
    wv_other = wv_min.clone()
    wv_max = jl.Vars.from_row(r30, now)
    wv_min.addPosition(10)
    wv_max.addPosition(30)
    wv_other.addPosition(30)
    wv_min.min(wv_other)
    assert (wv_min.posintext, wv_min.distance()) == (5, 5)
    wv_min.min(wv_other)
    assert (wv_min.posintext, wv_min.distance()) == (5, 5)
    wv_max.max(wv_other)
    assert (wv_max.posintext, wv_max.distance()) == (30, 25)
    wv_max.max(wv_other)
    wv_max.max(wv_other)
    assert (wv_max.posintext, wv_max.distance()) == (30, 25)
    wv_other.max(wv_max)
    assert (wv_other.posintext, wv_other.distance()) == (30, 25)


def test_referencecontainertest_add():
    """ReferenceContainerTest.testAdd (ReferenceContainerTest.java:51-100): the joined
    distance survives Vars -> 40-byte row -> Vars (J6 encodes distance() in column i)."""
    now = 20000 * jl.DAY
    v = jl.Vars.construct(b"kN0WkdoVHAAA", 25, 3, 0, 1, 1, 1, 1, [10], 1, 1, 0, b"en", ord("t"),
                          0, 0, jl.Bitfield(b"\0\0\0\0"), 0.0, now)
    assert v.distance() == 9
    back = jl.Vars.from_row(v.to_row(), now)
    assert back.distance() == v.distance() == 9


@pytest.mark.parametrize("n1,n2", [(1, 100), (100, 1), (2, 2), (1, 1), (50_000_000, 50_000_000),
                                   (37_000_000, 2_000_000), (1000, 1_000_000), (3, 3000),
                                   (2_147_483, 10), (53_687_091, 53_687_091)])
def test_dispatch_int_wrap(n1, n2):
    """J3: stepsEnum/stepsTest are Java ints and wrap (ReferenceContainer.java:406-409)."""
    assert orc.join_dispatch(n1, n2) == jl.join_dispatch(n1, n2)


def test_dispatch_wrap_flips_large_balanced_to_bytest():
    # 12*26*50M = 15.6e9 wraps negative -> stepsEnum > stepsTest -> by test
    assert jl.join_dispatch(50_000_000, 50_000_000)[0] is True
    assert jl.join_dispatch(20_000, 20_000)[0] is False


@pytest.mark.parametrize("sizes", [[5, 3, 9], [2_147_484, 10], [10, 2_147_484], [4_294_968, 1, 7],
                                   [1000, 1000, 1000], [0x7FFFFFFF // 1000 + 1, 5]])
def test_fold_order_int_wrap(sizes):
    """J2: TreeMap key (long)(int)(size*1000 + i) (ReferenceContainer.java:346)."""
    keys = {}
    for i, s in enumerate(sizes):
        keys[jl.i32(s * 1000 + i)] = i
    expect = [keys[k] for k in sorted(keys)]
    assert orc.fold_order(sizes) == expect


def test_profile_parse():
    rp = jl.RankingProfile.parse("", "{date=15,domlength=15,authority=13,tf=10}")
    assert (rp.coeff_date, rp.coeff_domlength, rp.coeff_authority, rp.coeff_termfrequency) == (15, 15, 13, 10)
    assert rp.coeff_posintext == 4  # defaults kept
    rp = jl.RankingProfile.parse("pre", "preDATE=3&predate=7&xx=1")
    assert rp.coeff_date == 7
    assert jl.parse_int_dec_substring("a=  -12x", 2) == -12


def _random_profile(rng):
    rp = jl.RankingProfile()
    for _, field in jl.PROFILE_FIELDS:
        setattr(rp, field, int(rng.integers(0, 16)))
    if rng.random() < 0.3:
        setattr(rp, "coeff_urlcomps", int(rng.integers(16, 40)))
    return rp


def _profiles():
    rng = np.random.default_rng(7)
    default = jl.RankingProfile()
    c5 = jl.RankingProfile.parse("", "date=15,domlength=15,authority=13,tf=10")
    date = jl.RankingProfile()
    date.all_zero()
    date.coeff_date = 15
    near = jl.RankingProfile()
    near.all_zero()
    near.coeff_worddistance = 15
    return [("default", default), ("c5", c5), ("date", date), ("near", near),
            ("rand1", _random_profile(rng)), ("rand2", _random_profile(rng))]


@pytest.mark.parametrize("preset,nq,minq,maxq,nexcl", [("dense", 12, 1, 4, 1), ("dense", 12, 2, 3, 0),
                                                       ("tiny", 12, 1, 2, 1)])
@pytest.mark.parametrize("today", [20741, 15500])
def test_literal_vs_cpp_random(preset, nq, minq, maxq, nexcl, today):
    """The object-level and the flat restatement agree on seeded synthetic data,
    including future dates (today=15500 puts part of the corpus in the future),
    multi-term folds (nonzero joined distances), exclusion, maxDistance and
    several ranking profiles."""
    cfg = synth.preset(preset)
    idx = synth.build_index(cfg)
    d = idx.as_dict()
    dl = {h: [bytes(r) for r in rows] for h, rows in d.items()}
    now = today * jl.DAY + 777
    qs = synth.queries(cfg, nq, minq, maxq, nexcl)
    nonempty = 0
    for qi, (inc, exc) in enumerate(qs):
        ih = [idx.hashes[t] for t in inc]
        eh = [idx.hashes[t] for t in exc]
        for md in (2147483647, 40):
            rows_l = jl.term_search(dl, ih, eh, md, now)
            rows_c = orc.term_search(d, ih, eh, md, now)
            assert b"".join(rows_l) == rows_c.tobytes(), (qi, md)
        for name, rp in _profiles()[: (6 if qi < 4 else 2)]:
            a = jl.search(dl, ih, eh, rp, "en", now_ms=now, k=100)
            b = [(h, s) for h, s, _ in orc.search(d, ih, eh, orc.profile_from(rp), "en", now_ms=now, k=100)]
            assert a == b, (qi, name)
            nonempty += bool(a)
    assert nonempty > 0


@pytest.mark.parametrize("frac", [0.01, 0.3])
def test_urlselection_restriction_is_the_literal_get(frac):
    """TermSearch's urlselection: the literal restatement of searchConjunction over
    ReferenceContainerCache.get(key, urlselection) (java_literal.term_search with a
    selection) equals the C++ oracle run over the lists restricted beforehand -- the
    restriction the GPU test (test_gpu_parity.test_urlselection_restricts_every_list)
    checks libyrwi against."""
    cfg = synth.preset("dense")
    idx = synth.build_index(cfg)
    d = idx.as_dict()
    dl = {h: [bytes(r) for r in rows] for h, rows in d.items()}
    urls = sorted({bytes(r[:12]) for r in np.asarray(idx.rows)})
    rng = np.random.default_rng(17)
    sel = {urls[i] for i in rng.choice(len(urls), max(1, int(frac * len(urls))), replace=False)}
    rd = {}
    for h, rows in d.items():
        keep = np.fromiter((bytes(r[:12]) in sel for r in rows), dtype=bool, count=len(rows))
        if keep.any():
            rd[h] = rows[keep]
    now = 20741 * jl.DAY + 5
    nonempty = 0
    for inc, exc in synth.queries(cfg, 16, 1, 4, 2, qseed=99):
        ih = [idx.hashes[t] for t in inc]
        eh = [idx.hashes[t] for t in exc]
        rows_l = jl.term_search(dl, ih, eh, 2147483647, now, urlselection=sel)
        rows_c = orc.term_search(rd, ih, eh, 2147483647, now)
        assert b"".join(rows_l) == rows_c.tobytes()
        nonempty += bool(rows_l)
    assert nonempty > 0
