"""Host-side mirror of YaCy's RWI query API over libyrwi (MI355X).

Mirrors the reference interface of the hot path so a caller written against
YaCy's classes finds the same names, argument meanings and "empty means no
result" behaviour (paths relative to /root/reference/source/net/yacy):

  RankingProfile           search/ranking/RankingProfile.java (defaults, external
                           string form, allZero)
  RWIIndex.add / get_size  kelondro/rwi/IndexCell.add (:289) / count
  RWIIndex.term_search     kelondro/rwi/TermSearch (:42-70) ->
                           ReferenceContainer.joinExcludeContainers (:310-326)
  ReferenceOrder           search/ranking/ReferenceOrder.normalizeWith (:70) +
                           cardinal (:223); settled (deterministic) min/max
  RWIIndex.search          SearchEvent.RWIProcess.run (:601-631) -> addRWIs
                           (:673-836) -> rwiStack top-k

All posting work runs in libyrwi's HIP kernels; this module only marshals.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import CFilter, CHit, CProfile, CQuery, CStats, YrwiError

INTEGER_MAX = 2147483647
MAX_RESULTS_RWI = 3000  # SearchEvent.java:118

# external attribute names (RankingProfile.java:42-75) -> coefficient field
_EXTERNAL = {
    "domlength": "coeff_domlength", "date": "coeff_date", "wordsintitle": "coeff_wordsintitle",
    "wordsintext": "coeff_wordsintext", "phrasesintext": "coeff_phrasesintext", "llocal": "coeff_llocal",
    "lother": "coeff_lother", "urllength": "coeff_urllength", "urlcomps": "coeff_urlcomps",
    "hitcount": "coeff_hitcount", "posintext": "coeff_posintext", "posofphrase": "coeff_posofphrase",
    "posinphrase": "coeff_posinphrase", "authority": "coeff_authority", "worddistance": "coeff_worddistance",
    "appurl": "coeff_appurl", "appdescr": "coeff_app_dc_title", "appauthor": "coeff_app_dc_creator",
    "apptags": "coeff_app_dc_subject", "appref": "coeff_app_dc_description", "appemph": "coeff_appemph",
    "catindexof": "coeff_catindexof", "cathasimage": "coeff_cathasimage", "cathasaudio": "coeff_cathasaudio",
    "cathasvideo": "coeff_cathasvideo", "cathasapp": "coeff_cathasapp", "tf": "coeff_termfrequency",
    "urlcompintoplist": "coeff_urlcompintoplist", "descrcompintoplist": "coeff_descrcompintoplist",
    "prefer": "coeff_prefer", "language": "coeff_language", "citation": "coeff_citation",
}


class RankingProfile:
    """search/ranking/RankingProfile.java.  Default = RankingProfile(ContentDomain.TEXT)."""

    COEFF_MIN = 0
    COEFF_MAX = 15

    def __init__(self, prefix: Optional[str] = None, profile: Optional[str] = None):
        self._c = CProfile()
        if profile:
            _lib.lib().yrwi_profile_parse((prefix or "").encode(), profile.encode(), ctypes.byref(self._c))
        else:
            _lib.lib().yrwi_profile_default(ctypes.byref(self._c))

    def __getattr__(self, name):
        if name.startswith("coeff_"):
            return getattr(self._c, name)
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name.startswith("coeff_"):
            setattr(self._c, name, int(value))
        else:
            object.__setattr__(self, name, value)

    def all_zero(self) -> "RankingProfile":  # allZero() :200-233
        _lib.lib().yrwi_profile_all_zero(ctypes.byref(self._c))
        return self

    @classmethod
    def date(cls) -> "RankingProfile":  # "/date" modifier, htroot/yacysearch.java:495-499
        p = cls().all_zero()
        p.coeff_date = cls.COEFF_MAX
        return p

    @classmethod
    def near(cls) -> "RankingProfile":  # "/near" modifier, htroot/yacysearch.java:489-494
        p = cls().all_zero()
        p.coeff_worddistance = cls.COEFF_MAX
        return p

    def to_external_map(self) -> dict:
        return {k: getattr(self._c, v) for k, v in _EXTERNAL.items()}

    @property
    def c(self) -> CProfile:
        return self._c


@dataclass
class Hit:
    urlhash: bytes
    score: int      # ReferenceOrder.cardinal
    tiebreak: int   # ByteArray.hashCode(urlhash)


class QueryFilter:
    """SearchEvent.addRWIs constraints (SearchEvent.java:736-806) and the doubledom
    pull order (pullOneRWI, :1297-1394); see yrwi_filter in include/yrwi.h.
    After a search, `flagcount` holds SearchEvent.flagcount (32 counters)."""

    def __init__(self, constraint: Optional[bytes] = None, all_of_constraint: bool = False, contentdom: int = 0,
                 strict_contentdom: bool = False, language: str = "", sitehash: Optional[bytes] = None,
                 alt_sitehash: Optional[bytes] = None, siteexcludes: Sequence[bytes] = (),
                 urlhashes: Sequence[bytes] = (), skip_double_dom: bool = False):
        c = CFilter()
        if constraint is not None:
            c.constraint[:] = list(bytes(constraint)[:4].ljust(4, b"\0"))
            c.has_constraint = 1
        c.all_of_constraint = int(all_of_constraint)
        c.contentdom = contentdom
        c.strict_contentdom = int(strict_contentdom)
        c.language = language.encode()[:7]
        if sitehash is not None:
            c.sitehash[:] = list(bytes(sitehash)[:6])
            c.has_sitehash = 1
        if alt_sitehash is not None:
            c.alt_sitehash[:] = list(bytes(alt_sitehash)[:6])
            c.has_alt_sitehash = 1
        sx = b"".join(bytes(h) for h in siteexcludes)
        uh = b"".join(bytes(h) for h in urlhashes)
        self._sx = ctypes.create_string_buffer(sx, max(1, len(sx)))
        self._uh = ctypes.create_string_buffer(uh, max(1, len(uh)))
        c.siteexcludes = ctypes.cast(self._sx, ctypes.c_void_p)
        c.nsiteexcludes = len(siteexcludes)
        c.urlhashes = ctypes.cast(self._uh, ctypes.c_void_p)
        c.nurlhashes = len(urlhashes)
        c.skip_double_dom = int(skip_double_dom)
        self._flags = (ctypes.c_int32 * 32)()
        c.flagcount = ctypes.cast(self._flags, ctypes.POINTER(ctypes.c_int32))
        self.c = c

    @property
    def flagcount(self) -> List[int]:
        return list(self._flags)


class SearchEvent:
    """One SearchEvent's RWI side (SearchEvent.addRWIs, SearchEvent.java:673-836):
    the local container and remote peers' containers (Protocol.java:802) arrive
    one after another; normalisation, doublecheck set, flag counts and the
    rwiStack persist on the GPU between arrivals (yrwi_event_* in include/yrwi.h)."""

    def __init__(self, index: "RWIIndex", profile: Optional[RankingProfile], language: str, now_ms: int, k: int,
                 filter: Optional[QueryFilter], max_postings: int, order_only_hosts: Optional[int] = None):
        self._ix = index
        self.k = k
        prof = profile or RankingProfile()
        e = ctypes.c_void_p()
        if order_only_hosts is not None:  # yrwi_event_open_order: order() / authority() only
            _check(index._h, _lib.lib().yrwi_event_open_order(index._h, ctypes.byref(prof._c), language.encode(),
                                                              now_ms, order_only_hosts, ctypes.byref(e)))
        else:
            fp = ctypes.byref(filter.c) if filter is not None else None
            _check(index._h, _lib.lib().yrwi_event_open(index._h, ctypes.byref(prof._c), language.encode(), now_ms, k,
                                                        fp, max_postings, ctypes.byref(e)))
        self._e = e

    def add_rwis(self, rows: np.ndarray, local: bool = False) -> int:
        return self._ix.add_rwis([(self, rows, local)])[0]

    def order(self, rows: np.ndarray, local: bool = False) -> np.ndarray:
        """ReferenceOrder.normalizeWith(container, local) + cardinal of every row
        (yrwi_event_order): the container continues the event's ReferenceOrder
        (min/max, max-distance fold, host counts over every container so far); the
        scores are under the state after it.  The stack is not touched: the
        drop-in's SearchEvent.addRWIs keeps its own (GpuReferenceOrder)."""
        r = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, 40)
        out = np.zeros(len(r), dtype=np.int64)
        if len(r):
            _check(self._ix._h, _lib.lib().yrwi_event_order(self._ix._h, self._e, r.ctypes.data, len(r),
                                                            int(bool(local)), out.ctypes.data))
        return out

    def authority(self, hosthashes: Sequence[bytes]) -> List[int]:
        """ReferenceOrder.authority(hostHash) against the accumulated host counts."""
        buf = b"".join(bytes(h)[:6] for h in hosthashes)
        out = (ctypes.c_int32 * max(1, len(hosthashes)))()
        if hosthashes:
            _check(self._ix._h, _lib.lib().yrwi_event_authority(self._ix._h, self._e, buf, len(hosthashes), out))
        return [int(out[i]) for i in range(len(hosthashes))]

    def source(self, urlhashes: Sequence[bytes]) -> List[Tuple[int, int]]:
        """(arrival, row) of each url's admitted posting (yrwi_event_source): arrival 1 is
        the event's first add_rwis arrival, 0 a seeded doublecheck url, -1 not admitted."""
        n = len(urlhashes)
        a = np.zeros(max(1, n), dtype=np.int32)
        r = np.zeros(max(1, n), dtype=np.int32)
        if n:
            _check(self._ix._h, _lib.lib().yrwi_event_source(self._ix._h, self._e, b"".join(bytes(u) for u in urlhashes),
                                                             n, a.ctypes.data, r.ctypes.data))
        return [(int(a[i]), int(r[i])) for i in range(n)]

    def results(self) -> Tuple[List["Hit"], "CEventInfo"]:
        out = (_lib.CHit * max(1, self.k))()
        n = ctypes.c_int32()
        info = _lib.CEventInfo()
        _check(self._ix._h, _lib.lib().yrwi_event_result(self._ix._h, self._e, out, self.k, ctypes.byref(n),
                                                         ctypes.byref(info)))
        return [Hit(bytes(out[i].urlhash), out[i].score, out[i].tiebreak) for i in range(n.value)], info

    def pull(self, n: int, skip_double_dom: bool = True) -> List["Hit"]:
        """SearchEvent.pullOneRWI(skipDoubleDom) up to n times (SearchEvent.java:1297-1394):
        the entries leave the stack; the doubleDomCache persists across calls."""
        out = (_lib.CHit * max(1, n))()
        got = ctypes.c_int32()
        _check(self._ix._h, _lib.lib().yrwi_event_pull(self._ix._h, self._e, 1 if skip_double_dom else 0, out, n,
                                                       ctypes.byref(got)))
        return [Hit(bytes(out[i].urlhash), out[i].score, out[i].tiebreak) for i in range(got.value)]

    def close(self):
        if self._e and self._ix._h:
            _lib.lib().yrwi_event_close(self._ix._h, self._e)
        self._e = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


@dataclass
class Query:
    include: Sequence[bytes]
    exclude: Sequence[bytes] = ()
    max_distance: int = INTEGER_MAX
    k: int = 100
    profile: Optional[RankingProfile] = None
    language: str = "en"
    now_ms: int = 0
    filter: Optional[QueryFilter] = None
    urlselection: Optional[Sequence[bytes]] = None  # TermSearch's urlselection (url hashes)


def _check(ctx, rc: int):
    if rc != 0:
        # ctx None: an open failed, and yrwi_last_error(NULL) holds this thread's reason
        msg = _lib.lib().yrwi_last_error(ctx)
        raise YrwiError(rc, (msg or b"").decode(errors="replace"))


def _hashes(hs: Sequence[bytes]) -> bytes:
    out = b"".join(bytes(h) for h in hs)
    if len(out) != 12 * len(hs):
        raise ValueError("term hashes must be 12 bytes")
    return out


class RWIIndex:
    """A device-resident reverse word index (one GPU, or one URL-hash shard).

    rows: numpy uint8 arrays of shape (n, 40) -- WordReferenceRow rows, i.e. the
    bytes of a RowSet chunkcache (RowCollection.java:68)."""

    def __init__(self, device: int = 0, shard: Optional[Tuple[int, int, bytes]] = None):
        L = _lib.lib()
        h = ctypes.c_void_p()
        if shard is None:
            _check(None, L.yrwi_open(device, ctypes.byref(h)))
        else:
            rank, world, uid = shard
            _check(None, L.yrwi_open_shard(device, rank, world, uid, ctypes.byref(h)))
        self._h = h
        self.device = device

    def shard_info(self) -> dict:
        """How this context's collectives travel (yrwi_shard_info): transport ("rccl",
        "host-staged", "loopback", "none"), RCCL communicator rank count, lanes, lanes
        with their own communicator, other ranks on this device, mailbox, PCI bus id."""
        info = _lib.CTransportInfo()
        _check(self._h, _lib.lib().yrwi_shard_info(self._h, ctypes.byref(info)))
        d = {f: getattr(info, f) for f, _ in _lib.CTransportInfo._fields_}
        d["transport"] = _lib.TRANSPORTS.get(d["transport"], str(d["transport"]))
        d["pci_bus_id"] = d["pci_bus_id"].decode(errors="replace")
        return d

    def close(self):
        if self._h:
            for p in getattr(self, "_pinned", []):
                _lib.lib().yrwi_host_free(self._h, p)
            self._pinned = []
            _lib.lib().yrwi_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- index maintenance (IndexCell) ----
    def add(self, term: bytes, rows: np.ndarray, sorted: bool = True) -> None:
        rows = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, 40)
        _check(self._h, _lib.lib().yrwi_put_list(self._h, bytes(term), rows.ctypes.data, len(rows), 1 if sorted else 0))

    def load_heaps(self, paths: Sequence[str], order_by_name: bool = False) -> "_lib.CLoadStats":
        """Load YaCy BLOB heap files (IndexCell's ReferenceContainerArray) into the index;
        lists already present act as the RAM cache (the files' rows win)."""
        arr = (ctypes.c_char_p * max(1, len(paths)))(*[p.encode() for p in paths])
        st = _lib.CLoadStats()
        _check(self._h, _lib.lib().yrwi_load_heaps(self._h, arr, len(paths), 1 if order_by_name else 0,
                                                   ctypes.byref(st)))
        return st

    def build_url_ids(self) -> None:
        """Bring the url dictionary up to date now (else the next query does)."""
        _check(self._h, _lib.lib().yrwi_build_url_ids(self._h))

    def check_url_ids(self) -> Tuple[int, int]:
        """(inconsistent postings / dictionary entries, dictionary size) after bringing
        the url ids up to date (diagnostic; 0 inconsistencies expected)."""
        bad, nurls = ctypes.c_int64(), ctypes.c_int64()
        _check(self._h, _lib.lib().yrwi_check_url_ids(self._h, ctypes.byref(bad), ctypes.byref(nurls)))
        return bad.value, nurls.value

    def index_info(self) -> dict:
        """Index maintenance counters (yrwi_index_info_get): dictionary full rebuilds /
        incremental updates, memory repacks, index arena bytes, bitmap lists."""
        info = _lib.CIndexInfo()
        _check(self._h, _lib.lib().yrwi_index_info_get(self._h, ctypes.byref(info)))
        return {f: getattr(info, f) for f, _ in _lib.CIndexInfo._fields_}

    def get_size(self, term: bytes) -> int:
        n = ctypes.c_int64()
        _check(self._h, _lib.lib().yrwi_list_size(self._h, bytes(term), ctypes.byref(n)))
        return n.value

    def get_list(self, term: bytes) -> np.ndarray:
        """Index.get(termHash) (AbstractIndex.java:116): the list's (n, 40) uint8 rows
        in url-hash order, (0, 40) when the term has no list (yrwi_get_list)."""
        n = self.get_size(term)
        out = np.zeros((max(n, 1), 40), dtype=np.uint8)
        m = ctypes.c_int64()
        _check(self._h, _lib.lib().yrwi_get_list(self._h, bytes(term), out.ctypes.data, n, ctypes.byref(m)))
        return out[:m.value]

    def stats(self) -> Tuple[int, int, int]:
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _check(self._h, _lib.lib().yrwi_index_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    # ---- TermSearch / joinExcludeContainers ----
    def term_search(self, include: Sequence[bytes], exclude: Sequence[bytes] = (),
                    max_distance: int = INTEGER_MAX, now_ms: int = 0,
                    urlselection: Optional[Sequence[bytes]] = None) -> np.ndarray:
        """The joined (and excluded) ReferenceContainer as (m, 40) uint8 rows
        (TermSearch.joined(); with `urlselection`, every list restricted to those urls)."""
        cap = 0
        for t in include:
            cap = max(cap, self.get_size(t))
        out = np.zeros((max(cap, 1), 40), dtype=np.uint8)
        m = ctypes.c_int64()
        if urlselection is None:
            _check(self._h, _lib.lib().yrwi_join_exclude(self._h, _hashes(include), len(include), _hashes(exclude),
                                                         len(exclude), max_distance, now_ms, out.ctypes.data, cap,
                                                         ctypes.byref(m)))
        else:
            arr, keep, _, _, _ = self._marshal([Query(include, exclude, max_distance, 1, None, "en", now_ms, None,
                                                      urlselection)], 1)
            _check(self._h, _lib.lib().yrwi_term_search(self._h, arr, out.ctypes.data, cap, ctypes.byref(m)))
        return out[:m.value].copy()

    # ---- ReferenceOrder.normalizeWith + cardinal ----
    def normalize_score(self, rows: np.ndarray, profile: Optional[RankingProfile] = None, language: str = "en",
                        now_ms: int = 0) -> np.ndarray:
        rows = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, 40)
        out = np.zeros(len(rows), dtype=np.int64)
        prof = profile or RankingProfile()
        _check(self._h, _lib.lib().yrwi_normalize_score(self._h, rows.ctypes.data, len(rows), ctypes.byref(prof.c),
                                                        language.encode(), now_ms, out.ctypes.data))
        return out

    # ---- search events: containers arriving one after another ----
    def event(self, profile: Optional[RankingProfile] = None, language: str = "en", now_ms: int = 0, k: int = 100,
              filter: Optional[QueryFilter] = None, max_postings: int = 1 << 16) -> "SearchEvent":
        return SearchEvent(self, profile, language, now_ms, k, filter, max_postings)

    def reference_order(self, profile: Optional[RankingProfile] = None, language: str = "en", now_ms: int = 0,
                        max_hosts: int = 1 << 16) -> "SearchEvent":
        """A SearchEvent's ReferenceOrder alone (yrwi_event_open_order, what
        GpuReferenceOrder holds): order() and authority(); no url set, no stack."""
        return SearchEvent(self, profile, language, now_ms, 1, None, 0, order_only_hosts=max_hosts)

    def add_rwis(self, arrivals: Sequence[Tuple["SearchEvent", np.ndarray, bool]]) -> List[int]:
        """Applies (event, rows (n, 40) uint8, local) arrivals in order, events in
        parallel (yrwi_event_add); returns the per-arrival codes (raises on the first
        error)."""
        arr = (_lib.CArrival * max(1, len(arrivals)))()
        keep = []
        for i, (ev, rows, local) in enumerate(arrivals):
            r = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, 40)
            keep.append(r)
            arr[i].ev = ev._e
            arr[i].rows40 = r.ctypes.data if len(r) else None
            arr[i].n = len(r)
            arr[i].local = int(bool(local))
        rc = _lib.lib().yrwi_event_add(self._h, arr, len(arrivals))
        codes = [arr[i].rc for i in range(len(arrivals))]
        _check(self._h, rc)
        return codes

    # ---- index abstracts (compressIndex) and the secondary search ----
    def index_abstracts(self, terms: Sequence[bytes], exclude: Optional[bytes] = None) -> List[bytes]:
        """searchConjunction + WordReferenceFactory.compressIndex per term; [] when
        a term has no list."""
        L = _lib.lib()
        sizes = [self.get_size(t) for t in terms]
        cap = sum(14 * n + 2 for n in sizes) + 2
        out = ctypes.create_string_buffer(max(1, cap))
        offs = (ctypes.c_int64 * (len(terms) + 1))()
        nout = ctypes.c_int32()
        _check(self._h, L.yrwi_index_abstracts(self._h, _hashes(terms), len(terms), exclude, out, cap, offs,
                                               ctypes.byref(nout)))
        raw = out.raw
        return [raw[offs[i]:offs[i + 1]] for i in range(nout.value)]

    def secondary_search(self, abstracts: Sequence[Tuple[bytes, bytes, bytes]], nwords_query: int, mypeer: bytes,
                         checked: Sequence[bytes] = (), decode: bool = True):
        """abstracts: (word, peer, text) in arrival order.  Returns (join [(url, peer)],
        words, plan [(peer, urls, words)]); with decode=False only (njoin, nplan)."""
        L = _lib.lib()
        arr = (_lib.CAbstract * max(1, len(abstracts)))()
        bufs = []
        total = 0
        for i, (w, p, t) in enumerate(abstracts):
            b = ctypes.create_string_buffer(bytes(t), max(1, len(t)))
            bufs.append(b)
            arr[i].word[:] = list(bytes(w))
            arr[i].peer[:] = list(bytes(p))
            arr[i].text = ctypes.cast(b, ctypes.c_void_p)
            arr[i].len = len(t)
            total += len(t)
        cap = total // 6 + 1
        ju = ctypes.create_string_buffer(12 * cap)
        jp = ctypes.create_string_buffer(12 * cap)
        pu = ctypes.create_string_buffer(12 * cap)
        plan = (_lib.CPeerRequest * max(1, len(abstracts)))()
        wo = ctypes.create_string_buffer(12 * 32)
        nj = ctypes.c_int64()
        npl = ctypes.c_int32()
        nw = ctypes.c_int32()
        _check(self._h, L.yrwi_secondary_search(self._h, arr, len(abstracts), nwords_query, bytes(mypeer),
                                                b"".join(bytes(c) for c in checked) or None, len(checked),
                                                ju, jp, cap, ctypes.byref(nj), plan, len(plan), ctypes.byref(npl),
                                                pu, wo, ctypes.byref(nw)))
        if not decode:
            return nj.value, npl.value
        wr, jur, jpr, pur = wo.raw, ju.raw, jp.raw, pu.raw  # each .raw is a copy: take them once
        words = [wr[12 * i:12 * i + 12] for i in range(nw.value)]
        join = [(jur[12 * i:12 * i + 12], jpr[12 * i:12 * i + 12]) for i in range(nj.value)]
        reqs = []
        for i in range(npl.value):
            r = plan[i]
            urls = [pur[12 * j:12 * j + 12] for j in range(r.url_off, r.url_off + r.url_n)]
            reqs.append((bytes(r.peer), urls, [words[b] for b in range(nw.value) if (r.words >> b) & 1]))
        return join, words, reqs

    # ---- ReferenceOrder.cardinal(URIMetadataNode): the Solr node stack ----
    def score_nodes(self, nodes: Sequence[dict], profile: Optional[RankingProfile] = None, language: str = "en",
                    maxdomcount: int = 0) -> np.ndarray:
        """nodes: dicts with urlhash, virtual_age, wordsintitle, wordcount, llocal, lother,
        flags (4 bytes), host_count, language (str or None) -- the URIMetadataNode fields
        cardinal reads (ReferenceOrder.java:267-296)."""
        n = len(nodes)
        arr = (_lib.CNode * max(1, n))()
        for i, d in enumerate(nodes):
            arr[i].urlhash[:] = list(bytes(d["urlhash"]))
            for f in ("virtual_age", "wordsintitle", "wordcount", "llocal", "lother", "host_count"):
                setattr(arr[i], f, int(d.get(f, 0)))
            arr[i].flags[:] = list(bytes(d.get("flags", b"\0\0\0\0"))[:4])
            arr[i].language = (d.get("language") or "").encode()[:7]
        out = np.zeros(max(1, n), dtype=np.int64)
        prof = profile or RankingProfile()
        _check(self._h, _lib.lib().yrwi_score_nodes(self._h, arr, n, ctypes.byref(prof._c), language.encode(),
                                                    maxdomcount, out.ctypes.data))
        return out[:n]

    # ---- full query: TermSearch -> normalise -> cardinal -> top-k ----
    def search(self, include: Sequence[bytes], exclude: Sequence[bytes] = (), profile: Optional[RankingProfile] = None,
               language: str = "en", max_distance: int = INTEGER_MAX, now_ms: int = 0, k: int = 100,
               stats: Optional[CStats] = None, filter: Optional[QueryFilter] = None) -> List[Hit]:
        return self.search_batch([Query(include, exclude, max_distance, k, profile, language, now_ms, filter)],
                                 stats=stats)[0]

    def _marshal(self, queries: Sequence[Query], kmax: Optional[int]):
        nq = len(queries)
        kmax = kmax or max(1, min(MAX_RESULTS_RWI, max(q.k for q in queries)))
        arr = (CQuery * nq)()
        keep = []
        for i, q in enumerate(queries):
            inc = _hashes(q.include)
            exc = _hashes(q.exclude)
            ib = ctypes.create_string_buffer(inc, max(1, len(inc)))
            eb = ctypes.create_string_buffer(exc, max(1, len(exc)))
            prof = q.profile or RankingProfile()
            keep += [ib, eb, prof]
            arr[i].incl = ctypes.cast(ib, ctypes.c_void_p)
            arr[i].nincl = len(q.include)
            arr[i].excl = ctypes.cast(eb, ctypes.c_void_p)
            arr[i].nexcl = len(q.exclude)
            arr[i].max_distance = q.max_distance
            arr[i].k = q.k
            arr[i].profile = ctypes.pointer(prof.c)
            arr[i].language = q.language.encode()[:7]
            arr[i].now_ms = q.now_ms
            if q.filter is not None:
                keep.append(q.filter)
                arr[i].filter = ctypes.pointer(q.filter.c)
            if q.urlselection is not None:
                sb = ctypes.create_string_buffer(_hashes(q.urlselection), max(1, 12 * len(q.urlselection)))
                keep.append(sb)
                arr[i].urlselection = ctypes.cast(sb, ctypes.c_void_p)
                arr[i].nurlselection = len(q.urlselection)
        hits = (CHit * (nq * kmax))()
        nout = (ctypes.c_int32 * nq)()
        return arr, keep, hits, nout, kmax

    @staticmethod
    def _unmarshal(nq: int, kmax: int, hits, nout) -> List[List[Hit]]:
        return [[Hit(bytes(hits[i * kmax + j].urlhash), hits[i * kmax + j].score, hits[i * kmax + j].tiebreak)
                 for j in range(nout[i])] for i in range(nq)]

    def search_batch(self, queries: Sequence[Query], stats: Optional[CStats] = None,
                     kmax: Optional[int] = None) -> List[List[Hit]]:
        nq = len(queries)
        if nq == 0:
            return []
        arr, keep, hits, nout, kmax = self._marshal(queries, kmax)
        st = stats if stats is not None else CStats()
        _check(self._h, _lib.lib().yrwi_query_batch(self._h, arr, nq, kmax, hits, nout, ctypes.byref(st)))
        return self._unmarshal(nq, kmax, hits, nout)

    def submit(self, queries: Sequence[Query], kmax: Optional[int] = None) -> "PendingBatch":
        """Start a batch asynchronously (yrwi_query_batch_submit); .result() waits for it.
        Batches run on the context's lanes in submission order (ticket t on lane t % lanes)."""
        nq = len(queries)
        arr, keep, hits, nout, kmax = self._marshal(queries, kmax) if nq else ((CQuery * 1)(), [], (CHit * 1)(),
                                                                               (ctypes.c_int32 * 1)(), 1)
        st = CStats()
        ticket = self.submit_raw(arr, nq, kmax, hits, nout, st)
        return PendingBatch(self, ticket, nq, kmax, (arr, keep, hits, nout, st))

    def search_batch_raw(self, cq, nq: int, kmax: int, hits, nout, st) -> None:
        """Zero-marshalling batch call for benchmarks (pre-built ctypes arrays).
        st None: no statistics (yrwi_stats* NULL, no HIP events: the production call)."""
        _check(self._h, _lib.lib().yrwi_query_batch(self._h, cq, nq, kmax, hits, nout,
                                                    ctypes.byref(st) if st is not None else None))

    # ---- asynchronous batches (yrwi_query_batch_submit / _wait) ----
    def submit_raw(self, cq, nq: int, kmax: int, hits, nout, st) -> int:
        """Start a batch; the ctypes buffers must stay alive until wait(ticket)."""
        t = ctypes.c_int64()
        _check(self._h, _lib.lib().yrwi_query_batch_submit(self._h, cq, nq, kmax, hits, nout,
                                                           ctypes.byref(st) if st is not None else None,
                                                           ctypes.byref(t)))
        return t.value

    def wait(self, ticket: int) -> None:
        _check(self._h, _lib.lib().yrwi_query_batch_wait(self._h, ticket))

    def host_array(self, ctype, n: int):
        """A ctypes array of n `ctype` in pinned host memory (GPU writes results into it directly)."""
        p = ctypes.c_void_p()
        _check(self._h, _lib.lib().yrwi_host_alloc(self._h, ctypes.sizeof(ctype) * max(1, n), ctypes.byref(p)))
        arr = (ctype * max(1, n)).from_address(p.value)
        self._pinned = getattr(self, "_pinned", []) + [p.value]
        return arr


class PendingBatch:
    """A submitted batch: its ctypes buffers stay alive until result() collects it."""

    def __init__(self, index: RWIIndex, ticket: int, nq: int, kmax: int, bufs):
        self.index, self.ticket, self.nq, self.kmax, self._bufs = index, ticket, nq, kmax, bufs

    def result(self) -> List[List[Hit]]:
        self.index.wait(self.ticket)
        _, _, hits, nout, _ = self._bufs
        return RWIIndex._unmarshal(self.nq, self.kmax, hits, nout)


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(None, _lib.lib().yrwi_get_unique_id(buf))
    return buf.raw
