"""Object-level restatement of YaCy's RWI query hot path (TEST INFRASTRUCTURE).

This module is part of the parity oracle.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it;
the product path (``yacy_search_server_amd``) never does.

It is a deliberately *literal* restatement: the classes and methods below keep
the shape of the Java classes they restate, so every line can be audited
against the reference.  It is slow (pure Python) and meant for small cases;
``oracle/yrwi_oracle.cpp`` is the fast restatement used as CPU baseline, and
the tests cross-check the two.

Reference files (paths relative to /root/reference/source/net/yacy):
  kelondro/data/word/WordReferenceRow.java     row layout :49-72, ctor :116-161
  kelondro/data/word/WordReferenceVars.java    Vars :78-158, clone :188-209,
                                               distance :287-294, toRowEntry
                                               :301-322, virtualAge :357-361,
                                               termFrequency :374-377,
                                               min :383-418, max :420-455,
                                               join :465-499, addPosition :534
  kelondro/rwi/AbstractReference.java          distance() :40-60
  kelondro/rwi/ReferenceContainer.java         joinExcludeContainers :310-326,
                                               joinContainers :328-371,
                                               excludeContainers :373-388,
                                               log2 :391-395, joinConstructive
                                               :397-417, ByTest :419-446,
                                               ByEnumeration :448-489,
                                               excludeDestructive :491-571
  kelondro/rwi/AbstractIndex.java              searchConjunction :96-128
  kelondro/rwi/TermSearch.java                 :42-70
  search/ranking/ReferenceOrder.java           NormalizeWorker :163-210,
                                               authority :213-216,
                                               cardinal :223-265
  search/ranking/RankingProfile.java           defaults :90-125, parse
                                               :127-194, allZero :200-233
  cora/sorting/WeakPriorityBlockingQueue.java  put :119-134, ReverseElement
                                               :400-426
  cora/util/ByteArray.java                     hashCode :80-84
  cora/date/MicroDate.java                     :37-55
  cora/order/Base64Order.java                  alphabet :38, compare :533-553
  cora/document/id/DigestURL.java              domLength :352-374
  kelondro/util/Bitfield.java                  get :88-93
  document/Tokenizer.java                      flags :51-56
  cora/util/NumberTools.java                   parseIntDecSubstring :91-124

Deterministic ("canonical") reading of the racy reference:
normalisation folds the container in ascending URL-hash order, ``cardinal`` is
evaluated against the settled min/max, no time limits apply, and "now" is an
explicit argument (``now_ms``) instead of System.currentTimeMillis().
"""

from __future__ import annotations

import bisect
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

# ---------------------------------------------------------------------------
# Java primitive semantics
# ---------------------------------------------------------------------------


def i32(x: int) -> int:
    """Java int wrap-around."""
    x &= 0xFFFFFFFF
    return x - 0x100000000 if x & 0x80000000 else x


def i64(x: int) -> int:
    """Java long wrap-around."""
    x &= 0xFFFFFFFFFFFFFFFF
    return x - 0x10000000000000000 if x & 0x8000000000000000 else x


def ishl(x: int, n: int) -> int:
    """Java ``int << n`` (shift count masked with 31)."""
    return i32(x << (n & 31))


def idiv(a: int, b: int) -> int:
    """Java int division, truncating toward zero (b != 0)."""
    q = abs(a) // abs(b)
    q = q if (a >= 0) == (b >= 0) else -q
    return i32(q)


def d2i(d: float) -> int:
    """Java (int) cast of a double."""
    if d != d:
        return 0
    if d >= 2147483647.0:
        return 2147483647
    if d <= -2147483648.0:
        return -2147483648
    return int(d)  # truncation toward zero


# ---------------------------------------------------------------------------
# Base64Order (enhancedCoder) and key helpers
# ---------------------------------------------------------------------------

ALPHA = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
AHPLA = [-1] * 128
for _i, _c in enumerate(ALPHA):
    AHPLA[_c] = _i


def wellformed(h: bytes) -> bool:
    return all(b < 128 and AHPLA[b] >= 0 for b in h)


def key72(h: bytes) -> int:
    """12 Base64 chars -> 72-bit integer whose order equals Base64Order.compare."""
    k = 0
    for b in h:
        k = (k << 6) | AHPLA[b]
    return k


def key_to_hash(k: int) -> bytes:
    return bytes(ALPHA[(k >> (6 * (11 - j))) & 63] for j in range(12))


def bytearray_hashcode(b: bytes) -> int:
    """ByteArray.hashCode(byte[]) (ByteArray.java:80-84)."""
    h = 0
    for c in b:
        h = i32(31 * h + (c & 0xFF))
    return h


# ---------------------------------------------------------------------------
# MicroDate (MicroDate.java:37-55)
# ---------------------------------------------------------------------------

DAY = 86400000


def micro_date_days(modified_ms: int) -> int:
    # (int) ((modified / day) % 262144L) with Java long division semantics
    q = abs(modified_ms) // DAY
    q = q if modified_ms >= 0 else -q
    r = abs(q) % 262144
    r = r if q >= 0 else -r
    return i32(r)


def reverse_micro_date_days(days: int, now_ms: int) -> int:
    return min(now_ms, i64(days * DAY))


# ---------------------------------------------------------------------------
# WordReferenceRow: 40-byte posting (WordReferenceRow.java:49-72)
# ---------------------------------------------------------------------------

# column: (offset, width)
COL = {
    "h": (0, 12), "a": (12, 2), "s": (14, 2), "u": (16, 1), "w": (17, 2),
    "p": (19, 2), "d": (21, 1), "l": (22, 2), "x": (24, 1), "y": (25, 1),
    "m": (26, 1), "n": (27, 1), "g": (28, 1), "z": (29, 4), "c": (33, 1),
    "t": (34, 2), "r": (36, 1), "o": (37, 1), "i": (38, 1), "k": (39, 1),
}
ROW_SIZE = 40

FLAG_APP_DC_DESCRIPTION = 24
FLAG_APP_DC_TITLE = 25
FLAG_APP_DC_CREATOR = 26
FLAG_APP_DC_SUBJECT = 27
FLAG_APP_DC_IDENTIFIER = 28
FLAG_APP_EMPHASIZED = 29
FLAG_CAT_INDEXOF = 0
FLAG_CAT_HASIMAGE = 20
FLAG_CAT_HASAUDIO = 21
FLAG_CAT_HASVIDEO = 22
FLAG_CAT_HASAPP = 23


def col_long(row: bytes, c: str) -> int:
    """Row.Entry.getColLong for a b256 cardinal cell: unsigned big-endian."""
    off, w = COL[c]
    v = 0
    for b in row[off:off + w]:
        v = (v << 8) | b
    return v


def col_bytes(row: bytes, c: str) -> bytes:
    off, w = COL[c]
    return bytes(row[off:off + w])


def encode_long(v: int, width: int) -> bytes:
    """NaturalOrder.encodeLong: low `width` bytes of the two's complement value."""
    return bytes(((v >> (8 * (width - 1 - j))) & 0xFF) for j in range(width))


class JavaNPE(Exception):
    """The reference would throw a NullPointerException on this input."""


class Bitfield:
    def __init__(self, bb: bytes):
        self.bb = bytes(bb)

    def get(self, pos: int) -> bool:  # Bitfield.java:88-93
        slot = pos >> 3
        if slot >= len(self.bb):
            return False
        b = self.bb[slot]
        b = b - 256 if b >= 128 else b  # Java byte
        return (b & (1 << (pos % 8))) > 0


def lang_from_row(row: bytes) -> Optional[bytes]:
    """getColBytes(col_language, nullIfEmpty=true) -> ASCII.String round trip."""
    l = col_bytes(row, "l")
    if l == b"\x00\x00":
        return None
    return l


def make_row(urlhash: bytes, urllength: int, urlcomps: int, titlewordcount: int,
             hitcount: int, wordcount: int, phrasecount: int, posintext: int,
             posinphrase: int, posofphrase: int, lastmodified_ms: int, updatetime_ms: int,
             language: Optional[bytes], doctype: int, outlinks_same: int,
             outlinks_other: int, word_distance: int, flags: bytes) -> bytes:
    """WordReferenceRow 18-argument constructor (WordReferenceRow.java:116-161)."""
    mddlm = micro_date_days(lastmodified_ms)
    mddct = micro_date_days(updatetime_ms)
    out = bytearray(ROW_SIZE)

    def put(c, b):
        off, w = COL[c]
        b = bytes(b)
        if len(b) < w:
            b = b + bytes(w - len(b))
        out[off:off + w] = b[:w]

    put("h", urlhash)
    put("a", encode_long(mddlm, 2))
    put("s", encode_long(max(0, i32(mddlm + i32((mddct - mddlm) * 2))), 2))
    put("u", encode_long(titlewordcount, 1))
    put("w", encode_long(wordcount, 2))
    put("p", encode_long(phrasecount, 2))
    put("d", bytes([doctype & 0xFF]))
    put("l", language if (language is not None and len(language) == 2) else b"en")
    put("x", encode_long(outlinks_same, 1))
    put("y", encode_long(outlinks_other, 1))
    put("m", encode_long(urllength, 1))
    put("n", encode_long(urlcomps, 1))
    put("g", b"\x00")
    put("z", flags)
    put("c", encode_long(hitcount, 1))
    put("t", encode_long(posintext, 2))
    put("r", encode_long(posinphrase, 1))
    put("o", encode_long(posofphrase, 1))
    put("i", encode_long(word_distance, 1))
    put("k", b"\x00")
    return bytes(out)


# ---------------------------------------------------------------------------
# WordReferenceVars (WordReferenceVars.java)
# ---------------------------------------------------------------------------


class Vars:
    __slots__ = ("flags", "lastModified", "language", "urlHash", "type", "hitcount",
                 "llocal", "lother", "phrasesintext", "posintext", "posinphrase",
                 "posofphrase", "urlcomps", "urllength", "wordsintext", "wordsintitle",
                 "distance_", "virtualAge_", "positions", "termFrequency_", "now_ms")

    @staticmethod
    def from_row(row: bytes, now_ms: int) -> "Vars":
        """new WordReferenceVars(new WordReferenceRow(entry), local) (:129-158)."""
        v = Vars()
        v.now_ms = now_ms
        v.flags = Bitfield(col_bytes(row, "z"))
        v.lastModified = reverse_micro_date_days(col_long(row, "a"), now_ms)
        v.language = lang_from_row(row)
        v.urlHash = col_bytes(row, "h")
        v.type = row[COL["d"][0]]
        v.hitcount = row[COL["c"][0]]
        v.llocal = row[COL["x"][0]]
        v.lother = row[COL["y"][0]]
        v.phrasesintext = col_long(row, "p")
        v.positions = None  # WordReferenceRow.positions() is null
        v.distance_ = col_long(row, "i")
        v.posinphrase = row[COL["r"][0]]
        v.posintext = col_long(row, "t")
        v.posofphrase = row[COL["o"][0]]
        v.urlcomps = row[COL["n"][0]]
        v.urllength = row[COL["m"][0]]
        v.virtualAge_ = col_long(row, "a")  # WordReferenceRow.virtualAge()
        v.wordsintext = col_long(row, "w")
        v.wordsintitle = row[COL["u"][0]]
        # WordReferenceRow.termFrequency (WordReferenceRow.java:355-357)
        v.termFrequency_ = float(v.hitcount) / float(v.wordsintext + v.wordsintitle + 1)
        return v

    @staticmethod
    def construct(urlHash, urllength, urlcomps, wordsintitle, hitcount, wordsintext,
                  phrasesintext, posintext, positions, posinphrase, posofphrase,
                  lastModified, language, type_, llocal, lother, flags, termFrequency,
                  now_ms) -> "Vars":
        """18-argument constructor (WordReferenceVars.java:78-127)."""
        v = Vars()
        v.now_ms = now_ms
        v.flags = flags
        v.lastModified = lastModified
        v.language = language
        v.urlHash = urlHash
        v.type = type_
        v.hitcount = hitcount
        v.llocal = llocal
        v.lother = lother
        v.phrasesintext = phrasesintext
        v.positions = list(positions) if positions else None
        v.distance_ = 0
        v.posinphrase = posinphrase
        v.posintext = posintext
        v.posofphrase = posofphrase
        v.urlcomps = urlcomps
        v.urllength = urllength
        v.virtualAge_ = -1
        v.wordsintext = wordsintext
        v.wordsintitle = wordsintitle
        v.termFrequency_ = termFrequency
        return v

    def clone(self) -> "Vars":  # :188-209
        return Vars.construct(self.urlHash, self.urllength, self.urlcomps, self.wordsintitle,
                              self.hitcount, self.wordsintext, self.phrasesintext,
                              self.posintext, self.positions, self.posinphrase,
                              self.posofphrase, self.lastModified, self.language, self.type,
                              self.llocal, self.lother, self.flags, self.termFrequency_,
                              self.now_ms)

    # AbstractReference.distance (AbstractReference.java:40-60)
    def _abstract_distance(self) -> int:
        if not self.positions:
            return 0
        d = 0
        s0 = self.posintext
        for s1 in self.positions:
            if s0 > 0:
                d = i32(d + abs(s0 - s1))
            s0 = s1
        return 0 if d == 0 else idiv(d, len(self.positions))

    def distance(self) -> int:  # :287-294
        value = self._abstract_distance()
        if value == 0:
            value = self.distance_
        return value

    def virtualAge(self) -> int:  # :357-361
        if self.virtualAge_ > 0:
            return self.virtualAge_
        self.virtualAge_ = micro_date_days(self.lastModified)
        return self.virtualAge_

    def termFrequency(self) -> float:  # :374-377
        if self.termFrequency_ == 0.0:
            self.termFrequency_ = float(self.hitcount) / float(self.wordsintext + self.wordsintitle + 1)
        return self.termFrequency_

    def hosthash(self) -> bytes:
        return self.urlHash[6:12]

    def getLanguage(self) -> bytes:
        if self.language is None:
            raise JavaNPE("ASCII.getBytes(null language)")
        return self.language

    def addPosition(self, position: int) -> None:  # :534-537
        if self.positions is None and position > 0:
            self.positions = []
        if position > 0:
            self.positions.append(position)

    def min(self, other: "Vars") -> None:  # :383-418
        if self.hitcount > other.hitcount: self.hitcount = other.hitcount
        if self.llocal > other.llocal: self.llocal = other.llocal
        if self.lother > other.lother: self.lother = other.lother
        v = other.virtualAge()
        if self.virtualAge() > v: self.virtualAge_ = v
        if self.wordsintext > other.wordsintext: self.wordsintext = other.wordsintext
        if self.phrasesintext > other.phrasesintext: self.phrasesintext = other.phrasesintext
        if self.posintext > other.posintext: self.posintext = other.posintext
        if self.distance() > 0 or other.distance() > 0:
            odist = other.distance()
            dist = self.distance()
            if odist > 0 and odist < dist:
                self.positions = [i32(self.posintext + odist)]
        if self.posinphrase > other.posinphrase: self.posinphrase = other.posinphrase
        if self.posofphrase > other.posofphrase: self.posofphrase = other.posofphrase
        if self.lastModified > other.lastModified: self.lastModified = other.lastModified
        if self.urllength > other.urllength: self.urllength = other.urllength
        if self.urlcomps > other.urlcomps: self.urlcomps = other.urlcomps
        if self.wordsintitle > other.wordsintitle: self.wordsintitle = other.wordsintitle
        if self.termFrequency_ > other.termFrequency_: self.termFrequency_ = other.termFrequency_

    def max(self, other: "Vars") -> None:  # :420-455
        if self.hitcount < other.hitcount: self.hitcount = other.hitcount
        if self.llocal < other.llocal: self.llocal = other.llocal
        if self.lother < other.lother: self.lother = other.lother
        v = other.virtualAge()
        if self.virtualAge() < v: self.virtualAge_ = v
        if self.wordsintext < other.wordsintext: self.wordsintext = other.wordsintext
        if self.phrasesintext < other.phrasesintext: self.phrasesintext = other.phrasesintext
        if self.posintext < other.posintext: self.posintext = other.posintext
        if self.distance() > 0 or other.distance() > 0:
            odist = other.distance()
            dist = self.distance()
            if odist > 0 and odist > dist:
                self.positions = [i32(self.posintext + odist)]
        if self.posinphrase < other.posinphrase: self.posinphrase = other.posinphrase
        if self.posofphrase < other.posofphrase: self.posofphrase = other.posofphrase
        if self.lastModified < other.lastModified: self.lastModified = other.lastModified
        if self.urllength < other.urllength: self.urllength = other.urllength
        if self.urlcomps < other.urlcomps: self.urlcomps = other.urlcomps
        if self.wordsintitle < other.wordsintitle: self.wordsintitle = other.wordsintitle
        if self.termFrequency_ < other.termFrequency_: self.termFrequency_ = other.termFrequency_

    def join(self, oe: "Vars") -> None:  # :465-499 (oe may be a row-derived Vars)
        if self.posintext > 0 and oe.posintext > 0:
            if self.posintext > oe.posintext:
                self.addPosition(self.posintext)
                self.posintext = oe.posintext
            else:
                self.addPosition(oe.posintext)
        elif self.posintext == 0:
            self.posintext = oe.posintext
        oe_posofphrase = oe.posofphrase
        if self.posofphrase == oe_posofphrase:
            self.posinphrase = min(self.posinphrase, oe.posinphrase)
        elif self.posofphrase > oe_posofphrase:
            self.posofphrase = oe_posofphrase
            self.posinphrase = oe.posinphrase
        self.termFrequency_ = self.termFrequency_ + oe.termFrequency()
        self.wordsintext = max(self.wordsintext, oe.wordsintext)
        self.wordsintitle = max(self.wordsintitle, oe.wordsintitle)
        self.phrasesintext = max(self.phrasesintext, oe.phrasesintext)
        self.hitcount = max(self.hitcount, oe.hitcount)

    def to_row(self) -> bytes:  # toRowEntry :301-322
        if self.language is None:
            raise JavaNPE("ASCII.getBytes(null language) in toRowEntry")
        return make_row(self.urlHash, self.urllength, self.urlcomps, self.wordsintitle,
                        self.hitcount, self.wordsintext, self.phrasesintext, self.posintext,
                        self.posinphrase, self.posofphrase, self.lastModified, self.now_ms,
                        self.language, self.type, self.llocal, self.lother, self.distance(),
                        self.flags.bb)


# ---------------------------------------------------------------------------
# ReferenceContainer algebra (ReferenceContainer.java:310-571)
# A container is a list of 40-byte rows sorted ascending by url hash.
# ---------------------------------------------------------------------------


def log2(x: int) -> int:  # :391-395
    l = 0
    while x > 0:
        x >>= 1
        l += 1
    return l


def join_by_test(small: List[bytes], large: List[bytes], max_distance: int, now_ms: int) -> List[bytes]:
    """:419-446 -- note the self-join: the large row is joined with itself."""
    large_keys = [key72(r[:12]) for r in large]
    conj = []
    for row in small:
        k = key72(row[:12])
        j = bisect.bisect_left(large_keys, k)
        if j < len(large_keys) and large_keys[j] == k:
            ie2 = Vars.from_row(large[j], now_ms)
            ie1 = Vars.from_row(large[j], now_ms)  # factory.produceFast(ie2, true)
            ie1.join(ie2)
            if ie1.distance() <= max_distance:
                conj.append(ie1.to_row())
    return conj


def join_by_enumeration(i1: List[bytes], i2: List[bytes], max_distance: int, now_ms: int) -> List[bytes]:
    """:448-489 -- sorted merge; result = Vars(i1 row) joined with i2 row."""
    conj = []
    if not i1 or not i2:
        return conj
    p1 = p2 = 0
    while True:
        c = key72(i1[p1][:12]) - key72(i2[p2][:12])
        if c < 0:
            p1 += 1
            if p1 >= len(i1):
                break
        elif c > 0:
            p2 += 1
            if p2 >= len(i2):
                break
        else:
            ie1 = Vars.from_row(i1[p1], now_ms)
            ie1.join(Vars.from_row(i2[p2], now_ms))
            if ie1.distance() <= max_distance:
                conj.append(ie1.to_row())
            p1 += 1
            if p1 >= len(i1):
                break
            p2 += 1
            if p2 >= len(i2):
                break
    return conj


def join_dispatch(n1: int, n2: int) -> Tuple[bool, bool]:
    """joinConstructive dispatch (:406-416) with Java int wrap.

    Returns (by_test, small_is_i1)."""
    high = n1 if n1 > n2 else n2
    low = n2 if n1 > n2 else n1
    steps_enum = i32(10 * i32(high + low - 1))
    steps_test = i32(i32(12 * log2(high)) * low)
    if steps_enum > steps_test:
        return True, n1 < n2
    return False, False


def join_constructive(i1: Optional[List[bytes]], i2: Optional[List[bytes]], max_distance: int,
                      now_ms: int, trace: Optional[list] = None) -> Optional[List[bytes]]:
    if i1 is None or i2 is None:
        return None
    if not i1 or not i2:
        return None
    by_test, small_is_i1 = join_dispatch(len(i1), len(i2))
    if trace is not None:
        trace.append(("test" if by_test else "enum", len(i1), len(i2)))
    if by_test:
        if small_is_i1:
            return join_by_test(i1, i2, max_distance, now_ms)
        return join_by_test(i2, i1, max_distance, now_ms)
    return join_by_enumeration(i1, i2, max_distance, now_ms)


def join_containers(containers: Sequence[List[bytes]], max_distance: int, now_ms: int,
                    trace: Optional[list] = None) -> Optional[List[bytes]]:
    """:328-371.  `containers` in term-hash order (TreeMap values)."""
    tmap: Dict[int, List[bytes]] = {}
    for count, c in enumerate(containers):
        if c is None or len(c) == 0:
            return None
        tmap[i32(len(c) * 1000 + count)] = c  # TreeMap.put overwrites on equal key
    if not tmap:
        return None
    keys = sorted(tmap)
    result = tmap[keys[0]]
    for k in keys[1:]:
        if len(result) == 0:
            break
        result = join_constructive(result, tmap[k], max_distance, now_ms, trace)
        if result is None:
            result = []
    if len(result) == 0:
        return None
    return result


def exclude_destructive(pivot: Optional[List[bytes]], excl: Optional[List[bytes]]) -> Optional[List[bytes]]:
    """:491-571.  Both ByTest and ByEnumeration remove every pivot row whose url
    hash occurs in `excl`, keeping the pivot order (RowCollection.removeRow
    keepOrder=true)."""
    if pivot is None:
        return None
    if excl is None:
        return pivot
    if len(pivot) == 0:
        return None
    if len(excl) == 0:
        return pivot
    ex = set(r[:12] for r in excl)
    pivot[:] = [r for r in pivot if r[:12] not in ex]
    return pivot


def exclude_containers(pivot: List[bytes], containers: Sequence[List[bytes]]) -> Optional[List[bytes]]:
    if not containers:
        return pivot
    for c in containers:
        pivot = exclude_destructive(pivot, c)
        if pivot is None or len(pivot) == 0:
            return None
    return pivot


def term_search(index: Dict[bytes, List[bytes]], include: Iterable[bytes], exclude: Iterable[bytes],
                max_distance: int, now_ms: int, trace: Optional[list] = None,
                urlselection: Optional[Iterable[bytes]] = None) -> List[bytes]:
    """TermSearch.<init> (TermSearch.java:42-70) + AbstractIndex.searchConjunction
    (AbstractIndex.java:96-128) + joinExcludeContainers (:310-326).

    HandleSet semantics: term hashes are a sorted set (duplicates collapse).
    Returns a *new* list (the reference mutates the index container for
    one-term queries; we never mutate the index).  `urlselection` (url hashes):
    every container as ReferenceContainerCache.get(key, urlselection) returns it
    (ReferenceContainerCache.java:448-470): its entries whose url hash is in the
    selection, in order -- an empty one counts as missing in searchConjunction."""
    inc = sorted(set(include), key=lambda h: key72(h))
    exc = sorted(set(exclude), key=lambda h: key72(h))
    sel = None if urlselection is None else set(bytes(u) for u in urlselection)

    def get(h):
        c = index.get(h)
        if c is None or sel is None:
            return c
        return [r for r in c if bytes(r[:12]) in sel]

    def conjunction(hashes):
        out = []
        for h in hashes:
            c = get(h)
            if c is None or len(c) == 0:
                return []  # any missing term -> empty map
            out.append(list(c))
        return out

    inclusion = conjunction(inc) if inc else []
    exclusion = conjunction(exc) if inclusion else []
    if not inclusion:
        return []
    rc = join_containers(inclusion, max_distance, now_ms, trace)
    if rc is None:
        return []
    rc = list(rc)
    exclude_containers(rc, exclusion)
    return rc


# ---------------------------------------------------------------------------
# RankingProfile (RankingProfile.java)
# ---------------------------------------------------------------------------

PROFILE_FIELDS = [
    # (attribute name in external form, coefficient field)
    ("domlength", "coeff_domlength"), ("date", "coeff_date"),
    ("wordsintitle", "coeff_wordsintitle"), ("wordsintext", "coeff_wordsintext"),
    ("phrasesintext", "coeff_phrasesintext"), ("llocal", "coeff_llocal"),
    ("lother", "coeff_lother"), ("urllength", "coeff_urllength"),
    ("urlcomps", "coeff_urlcomps"), ("hitcount", "coeff_hitcount"),
    ("posintext", "coeff_posintext"), ("posofphrase", "coeff_posofphrase"),
    ("posinphrase", "coeff_posinphrase"), ("authority", "coeff_authority"),
    ("worddistance", "coeff_worddistance"), ("appurl", "coeff_appurl"),
    ("appdescr", "coeff_app_dc_title"), ("appauthor", "coeff_app_dc_creator"),
    ("apptags", "coeff_app_dc_subject"), ("appref", "coeff_app_dc_description"),
    ("appemph", "coeff_appemph"), ("catindexof", "coeff_catindexof"),
    ("cathasimage", "coeff_cathasimage"), ("cathasaudio", "coeff_cathasaudio"),
    ("cathasvideo", "coeff_cathasvideo"), ("cathasapp", "coeff_cathasapp"),
    ("tf", "coeff_termfrequency"), ("urlcompintoplist", "coeff_urlcompintoplist"),
    ("descrcompintoplist", "coeff_descrcompintoplist"), ("prefer", "coeff_prefer"),
    ("language", "coeff_language"), ("citation", "coeff_citation"),
]


class RankingProfile:
    def __init__(self):  # RankingProfile(ContentDomain.TEXT) :90-125
        self.coeff_appemph = 5
        self.coeff_appurl = 12
        self.coeff_app_dc_creator = 1
        self.coeff_app_dc_description = 10
        self.coeff_app_dc_subject = 2
        self.coeff_app_dc_title = 14
        self.coeff_authority = 5
        self.coeff_cathasapp = 0
        self.coeff_cathasaudio = 0
        self.coeff_cathasimage = 0
        self.coeff_cathasvideo = 0
        self.coeff_catindexof = 0
        self.coeff_date = 9
        self.coeff_domlength = 10
        self.coeff_hitcount = 1
        self.coeff_language = 2
        self.coeff_llocal = 0
        self.coeff_lother = 7
        self.coeff_phrasesintext = 0
        self.coeff_posinphrase = 0
        self.coeff_posintext = 4
        self.coeff_posofphrase = 0
        self.coeff_termfrequency = 8
        self.coeff_urlcomps = 7
        self.coeff_urllength = 6
        self.coeff_worddistance = 10
        self.coeff_wordsintext = 3
        self.coeff_wordsintitle = 2
        self.coeff_urlcompintoplist = 2
        self.coeff_descrcompintoplist = 2
        self.coeff_prefer = 0
        self.coeff_citation = 10

    @staticmethod
    def parse(prefix: Optional[str], profile: Optional[str]) -> "RankingProfile":
        """RankingProfile(String prefix, String profile) :127-189."""
        rp = RankingProfile()
        if profile is None or len(profile) == 0:
            return rp
        coeff: Dict[str, int] = {}
        if profile[0] == "{" and profile.endswith("}"):
            profile = profile[1:-1]
        profile = profile.strip()
        elts = profile.split("&") if profile.find("&") > 0 else profile.split(",")
        s = 0 if prefix is None else len(prefix)
        for elt in elts:
            e = elt.strip()
            if s == 0 or e.startswith(prefix):
                p = e.find("=")
                if p > 0 and len(e) > p + 1:
                    try:
                        coeff[e[s:p]] = parse_int_dec_substring(e, p + 1)
                    except ValueError:
                        pass
        for name, field in PROFILE_FIELDS:
            if name in coeff:
                setattr(rp, field, coeff[name])
        return rp

    def all_zero(self) -> None:  # :200-233
        for _, field in PROFILE_FIELDS:
            setattr(self, field, 0)


def parse_int_dec_substring(s: str, start: int) -> int:
    """NumberTools.parseIntDecSubstring (NumberTools.java:91-124)."""
    end = len(s)
    if end <= start:
        raise ValueError(s)
    i = start
    while s[i] == " ":
        i += 1
    result = 0
    negative = False
    limit = -2147483647
    first = s[i]
    if first < "0":
        if first == "-":
            negative = True
            limit = -2147483648
        elif first != "+":
            raise ValueError(s)
        i += 1
        if i == end:
            raise ValueError(s)
    multmin = int(limit / 10)
    while i < end:
        c = s[i]
        i += 1
        if c < "0" or c > "9":
            break
        digit = ord(c) - 48
        if result < multmin:
            raise ValueError(s)
        result *= 10
        if result < limit + digit:
            raise ValueError(s)
        result -= digit
    return result if negative else -result


# ---------------------------------------------------------------------------
# ReferenceOrder (ReferenceOrder.java)
# ---------------------------------------------------------------------------


def dom_length_normalized(urlhash: bytes) -> int:
    """DigestURL.domLengthNormalized (:352-374): x << (8 / 20) == x << 0."""
    flagbyte = AHPLA[urlhash[11]]
    key = flagbyte & 3
    return {0: 4, 1: 10, 2: 14, 3: 20}[key] << (8 // 20)


class ReferenceOrder:
    def __init__(self, profile: RankingProfile, language: str):
        self.min: Optional[Vars] = None
        self.max: Optional[Vars] = None
        self.ranking = profile
        self.doms: Dict[bytes, int] = {}
        self.maxdomcount = 0
        self.language = language

    def normalize_with(self, container: List[bytes], now_ms: int) -> List[Vars]:
        """Canonical single-worker NormalizeWorker.run (:163-210)."""
        out = []
        for row in container:
            e = Vars.from_row(row, now_ms)
            if self.min is None:
                self.min = e.clone()
            else:
                self.min.min(e)
            if self.max is None:
                self.max = e.clone()
            else:
                self.max.max(e)
            out.append(e)
            d = e.hosthash()
            self.doms[d] = self.doms.get(d, 0) + 1
        if self.doms:
            self.maxdomcount = max(self.doms.values())
        return out

    def authority(self, hosthash: bytes) -> int:  # :213-216
        return idiv(ishl(self.doms.get(hosthash, 0), 8), i32(1 + self.maxdomcount))

    def cardinal(self, t: Vars) -> int:  # :223-265
        mn, mx, rk = self.min, self.max, self.ranking
        flags = t.flags
        if mx.termFrequency() == mn.termFrequency():
            tf = 0
        else:
            tf = ishl(d2i(((t.termFrequency() - mn.termFrequency()) * 256.0)
                          / (mx.termFrequency() - mn.termFrequency())), rk.coeff_termfrequency)

        def inv(tv, lo, hi, coeff):  # (max == min) ? 0 : (256 - ((t - min) << 8) / (max - min)) << coeff
            if hi == lo:
                return 0
            return ishl(i32(256 - idiv(ishl(i32(tv - lo), 8), i32(hi - lo))), coeff)

        def fwd(tv, lo, hi, coeff):  # (max == min) ? 0 : (((t - min) << 8) / (max - min)) << coeff
            if hi == lo:
                return 0
            return ishl(idiv(ishl(i32(tv - lo), 8), i32(hi - lo)), coeff)

        r = ishl(256 - dom_length_normalized(t.urlHash), rk.coeff_domlength)
        r = i32(r + inv(t.urlcomps, mn.urlcomps, mx.urlcomps, rk.coeff_urlcomps))
        r = i32(r + inv(t.urllength, mn.urllength, mx.urllength, rk.coeff_urllength))
        r = i32(r + inv(t.posintext, mn.posintext, mx.posintext, rk.coeff_posintext))
        r = i32(r + inv(t.posofphrase, mn.posofphrase, mx.posofphrase, rk.coeff_posofphrase))
        r = i32(r + inv(t.posinphrase, mn.posinphrase, mx.posinphrase, rk.coeff_posinphrase))
        r = i32(r + inv(t.distance(), mn.distance(), mx.distance(), rk.coeff_worddistance))
        r = i32(r + fwd(t.virtualAge(), mn.virtualAge(), mx.virtualAge(), rk.coeff_date))
        r = i32(r + fwd(t.wordsintitle, mn.wordsintitle, mx.wordsintitle, rk.coeff_wordsintitle))
        r = i32(r + fwd(t.wordsintext, mn.wordsintext, mx.wordsintext, rk.coeff_wordsintext))
        r = i32(r + fwd(t.phrasesintext, mn.phrasesintext, mx.phrasesintext, rk.coeff_phrasesintext))
        r = i32(r + fwd(t.llocal, mn.llocal, mx.llocal, rk.coeff_llocal))
        r = i32(r + fwd(t.lother, mn.lother, mx.lother, rk.coeff_lother))
        r = i32(r + fwd(t.hitcount, mn.hitcount, mx.hitcount, rk.coeff_hitcount))
        # + tf switches the accumulation to long
        R = i64(r + tf)
        R = i64(R + (ishl(self.authority(t.hosthash()), rk.coeff_authority) if rk.coeff_authority > 12 else 0))
        for bit, coeff in ((FLAG_APP_DC_IDENTIFIER, rk.coeff_appurl),
                           (FLAG_APP_DC_TITLE, rk.coeff_app_dc_title),
                           (FLAG_APP_DC_CREATOR, rk.coeff_app_dc_creator),
                           (FLAG_APP_DC_SUBJECT, rk.coeff_app_dc_subject),
                           (FLAG_APP_DC_DESCRIPTION, rk.coeff_app_dc_description),
                           (FLAG_APP_EMPHASIZED, rk.coeff_appemph),
                           (FLAG_CAT_INDEXOF, rk.coeff_catindexof),
                           (FLAG_CAT_HASIMAGE, rk.coeff_cathasimage),
                           (FLAG_CAT_HASAUDIO, rk.coeff_cathasaudio),
                           (FLAG_CAT_HASVIDEO, rk.coeff_cathasvideo),
                           (FLAG_CAT_HASAPP, rk.coeff_cathasapp)):
            R = i64(R + (ishl(255, coeff) if flags.get(bit) else 0))
        target = self.language.encode("latin-1")
        R = i64(R + (ishl(255, rk.coeff_language) if t.getLanguage() == target else 0))
        return R


# ---------------------------------------------------------------------------
# WeakPriorityBlockingQueue with ReverseElement (WeakPriorityBlockingQueue.java)
# ---------------------------------------------------------------------------


def cardinal_node(order: "ReferenceOrder", urlhash: bytes, virtual_age: int, wordsintitle: int, wordcount: int,
                  llocal: int, lother: int, flags: bytes, language: Optional[str]) -> int:
    """ReferenceOrder.cardinal(URIMetadataNode) (ReferenceOrder.java:267-296): the
    Solr node stack's fallback score.  Every term is a Java int, so the sum wraps
    as an int before it is widened to long; `language` None is a node without a
    language (String.equals(null) is false).  The authority term uses the order's
    host counts (ReferenceOrder.authority :213-216)."""
    rk = order.ranking
    f = Bitfield(flags)
    terms = [
        ishl(256 - dom_length_normalized(urlhash), rk.coeff_domlength),
        ishl(virtual_age, rk.coeff_date),
        ishl(wordsintitle, rk.coeff_wordsintitle),
        ishl(wordcount, rk.coeff_wordsintext),
        ishl(llocal, rk.coeff_llocal),
        ishl(lother, rk.coeff_lother),
        ishl(order.authority(urlhash[6:12]), rk.coeff_authority) if rk.coeff_authority > 12 else 0,
        ishl(255, rk.coeff_appurl) if f.get(FLAG_APP_DC_IDENTIFIER) else 0,
        ishl(255, rk.coeff_app_dc_title) if f.get(FLAG_APP_DC_TITLE) else 0,
        ishl(255, rk.coeff_app_dc_creator) if f.get(FLAG_APP_DC_CREATOR) else 0,
        ishl(255, rk.coeff_app_dc_subject) if f.get(FLAG_APP_DC_SUBJECT) else 0,
        ishl(255, rk.coeff_app_dc_description) if f.get(FLAG_APP_DC_DESCRIPTION) else 0,
        ishl(255, rk.coeff_appemph) if f.get(FLAG_APP_EMPHASIZED) else 0,
        ishl(255, rk.coeff_catindexof) if f.get(FLAG_CAT_INDEXOF) else 0,
        ishl(255, rk.coeff_cathasimage) if f.get(FLAG_CAT_HASIMAGE) else 0,
        ishl(255, rk.coeff_cathasaudio) if f.get(FLAG_CAT_HASAUDIO) else 0,
        ishl(255, rk.coeff_cathasvideo) if f.get(FLAG_CAT_HASVIDEO) else 0,
        ishl(255, rk.coeff_cathasapp) if f.get(FLAG_CAT_HASAPP) else 0,
        ishl(255, rk.coeff_language) if (language is not None and order.language == language) else 0,
    ]
    r = 0
    for t in terms:
        r = i32(r + t)
    return r


class ReverseQueue:
    """Bounded TreeSet ordered by ReverseElement.compareTo (:414-425)."""

    def __init__(self, maxsize: int):
        self.maxsize = maxsize
        self.items: List[Tuple[int, int, bytes]] = []  # (weight, hash, urlhash) best first

    @staticmethod
    def _cmp(a, b) -> int:
        if a[2] == b[2]:
            return 0
        if a[0] > b[0]:
            return -1
        if a[0] < b[0]:
            return 1
        if a[1] > b[1]:
            return -1
        if a[1] < b[1]:
            return 1
        return 0

    def _add(self, e) -> bool:
        lo, hi = 0, len(self.items)
        while lo < hi:
            mid = (lo + hi) // 2
            c = self._cmp(e, self.items[mid])
            if c == 0:
                return False
            if c < 0:
                hi = mid
            else:
                lo = mid + 1
        # TreeSet rejects any element comparing equal to an existing one; the
        # binary search above only meets one candidate, so check neighbours too.
        for j in (lo - 1, lo):
            if 0 <= j < len(self.items) and self._cmp(e, self.items[j]) == 0:
                return False
        self.items.insert(lo, e)
        return True

    def put(self, weight: int, urlhash: bytes) -> None:  # :119-134
        e = (weight, bytearray_hashcode(urlhash), urlhash)
        if len(self.items) == self.maxsize:
            if self._add(e):
                self.items.pop()
        else:
            self._add(e)


MAX_RESULTS_RWI = 3000  # SearchEvent.java:118


class QueryFilter:
    """The per-query constraints addRWIs applies before a posting enters rwiStack
    (SearchEvent.java:736-806) and the doubledom pull order (:1297-1394).
    Defaults reproduce the unconstrained query."""

    def __init__(self, constraint: Optional[bytes] = None, all_of_constraint: bool = False, contentdom: int = 0,
                 strict_contentdom: bool = False, language: str = "", sitehash: Optional[bytes] = None,
                 alt_sitehash: Optional[bytes] = None, siteexcludes: Sequence[bytes] = (),
                 urlhashes: Sequence[bytes] = (), skip_double_dom: bool = False):
        self.constraint = Bitfield(constraint) if constraint is not None else None  # QueryParams.constraint
        self.all_of_constraint = all_of_constraint
        self.contentdom = contentdom          # ContentDomain code (Classification.java:47-52)
        self.strict_contentdom = strict_contentdom
        self.language = language              # QueryModifier.language
        self.sitehash = sitehash              # QueryModifier.sitehash
        self.alt_sitehash = alt_sitehash      # acceptableAlternativeSitehash (:716-718)
        self.siteexcludes = set(siteexcludes)
        self.urlhashes = set(urlhashes)       # SearchEvent.urlhashes (doublecheck)
        self.skip_double_dom = skip_double_dom
        self.flagcount = [0] * 32             # SearchEvent.flagcount

    def test_flags(self, flags: Bitfield) -> bool:  # SearchEvent.testFlags :2459-2474
        if self.constraint is None:
            return True
        if self.all_of_constraint:
            for i in range(32):
                if self.constraint.get(i) and not flags.get(i):
                    return False
            return True
        for i in range(32):
            if self.constraint.get(i) and flags.get(i):
                return True
        return False

    def admit(self, e: "Vars") -> bool:
        """addRWIs pollloop body up to rwiStack.put (:736-806); True = put on the stack."""
        if e.urlHash in self.urlhashes:       # doublecheck (:736-740)
            return False
        flags = e.flags
        for j in range(32):                   # flag counts (:743-746)
            if flags.get(j):
                self.flagcount[j] += 1
        if not self.test_flags(flags):        # (:749-752)
            return False
        if self.contentdom > 0:               # (:755-775), Tokenizer flags :51-56, Response.DT_*
            t = chr(e.type)
            if self.strict_contentdom:
                bad = ((self.contentdom == 2 and t != "a") or (self.contentdom == 3 and t != "m") or
                       (self.contentdom == 1 and t != "i") or (self.contentdom == 4 and not flags.get(23)))
            else:
                bad = ((self.contentdom == 2 and not flags.get(21)) or (self.contentdom == 3 and not flags.get(22)) or
                       (self.contentdom == 1 and not flags.get(20)) or (self.contentdom == 4 and not flags.get(23)))
            if bad:
                return False
        if self.language:                      # (:778-784): modifier.language.equals(getLanguageString())
            lang = e.language.decode("latin-1") if e.language is not None else None
            if self.language != lang:
                return False
        h = e.hosthash()                       # (:790-802)
        if self.sitehash is None:
            if h in self.siteexcludes:
                return False
        elif h != self.sitehash and (self.alt_sitehash is None or h != self.alt_sitehash):
            return False
        self.urlhashes.add(e.urlHash)          # urlhashes.putUnique (:805)
        return True


def pull_double_dom(items: List[Tuple[bytes, int]], n: int) -> List[Tuple[bytes, int]]:
    """pullOneRWI(skipDoubleDom = true) repeated n times over a settled rwiStack
    (SearchEvent.java:1297-1394).  items: the stack, best first.  Each round polls
    at most 10 stack entries; the first whose host has no doubleDomCache entry is
    returned (and creates one), the others go to their host's queue.  If none was
    returned, the best head of the host queues is returned and a host whose queue
    becomes empty leaves the cache.  The reference picks that head by weight over
    a ConcurrentHashMap walk; equal weights are resolved here by stack position
    (the earliest queued entry), which is the best head under the stack order."""
    out: List[Tuple[bytes, int]] = []
    cache: Dict[bytes, List[int]] = {}  # host -> queued stack positions
    queued: List[int] = []              # all queued positions, in push order (= stack order)
    i = 0
    while len(out) < n:
        c = 0
        got = None
        while i < len(items) and c < 10:
            pos = i
            i += 1
            c += 1
            h = items[pos][0][6:12]
            if h not in cache:
                cache[h] = []
                got = pos
                break
            cache[h].append(pos)
            queued.append(pos)
        if got is not None:
            out.append(items[got])
            continue
        if not cache or not queued:
            break
        pos = queued.pop(0)
        h = items[pos][0][6:12]
        cache[h].remove(pos)
        if not cache[h]:
            del cache[h]
        out.append(items[pos])
    return out


def rank(container: List[bytes], profile: RankingProfile, language: str, now_ms: int,
         maxsize: int = MAX_RESULTS_RWI, filt: Optional[QueryFilter] = None) -> List[Tuple[bytes, int]]:
    """normalizeWith + addRWIs poll loop (SearchEvent.java:697-816).  Without
    `filt` the query is unconstrained (no doublecheck hits, no constraint /
    contentdom / language / site filter).  Normalisation covers the whole
    container; the filters only decide what enters the stack."""
    if not container:
        return []
    order = ReferenceOrder(profile, language)
    entries = order.normalize_with(container, now_ms)
    q = ReverseQueue(maxsize)
    for e in entries:
        if filt is not None and not filt.admit(e):
            continue
        q.put(order.cardinal(e), e.urlHash)
    return [(h, w) for (w, _, h) in q.items]


class SearchEventRWI:
    """The RWI side of one SearchEvent fed container by container
    (SearchEvent.addRWIs :673-836, called by RWIProcess.run :612-631 for the
    local container and by Protocol.remoteSearchProcess :802 for every remote
    peer).  The ReferenceOrder (min/max, distance fold, doms), the doublecheck
    set, the flag counts and rwiStack persist between calls; each arrival is
    normalised completely before its entries are scored (the canonical settled
    order of DESIGN.md §2, per arrival), so entries keep the score they got when
    they arrived."""

    def __init__(self, profile: RankingProfile, language: str, now_ms: int,
                 filt: Optional[QueryFilter] = None, maxsize: int = MAX_RESULTS_RWI):
        self.order = ReferenceOrder(profile, language)
        self.filt = filt if filt is not None else QueryFilter()
        self.now_ms = now_ms
        self.q = ReverseQueue(maxsize)
        self.local_available = 0
        self.remote_available = 0
        self.remote_peers = 0

    def add_rwis(self, container: List[bytes], local: bool) -> int:
        if not container:                      # index.isEmpty() -> return 0 (:685)
            return 0
        if not local:
            self.remote_peers += 1
        entries = self.order.normalize_with(container, self.now_ms)
        n = 0
        for e in entries:
            if not self.filt.admit(e):
                continue
            self.q.put(self.order.cardinal(e), e.urlHash)
            n += 1
        if local:
            self.local_available += n
        else:
            self.remote_available += n
        return n

    def stack(self) -> List[Tuple[bytes, int]]:
        return [(h, w) for (w, _, h) in self.q.items]

    def pull(self, n: int, skip_double_dom: bool) -> List[Tuple[bytes, int]]:
        """pullOneRWI(skipDoubleDom) (SearchEvent.java:1297-1394) up to n times,
        stopping at the first null; polled entries leave rwiStack and the
        doubleDomCache persists between calls (arrivals may come in between).
        The metadata lookup (:1309,1327,1392) is outside the RWI path: every url
        is taken to have metadata."""
        if not hasattr(self, "dd"):
            self.dd: Dict[bytes, ReverseQueue] = {}   # doubleDomCache (:426)
            self.dd_seq: Dict[bytes, int] = {}        # url -> when it was queued
            self.dd_next = 0
        out: List[Tuple[bytes, int]] = []
        while len(out) < n:
            e = self._pull_one(skip_double_dom)
            if e is None:
                break
            out.append(e)
        return out

    def _pull_one(self, skip: bool) -> Optional[Tuple[bytes, int]]:
        c = 0
        while len(self.q.items) > 0 and c < 10:        # pollloop (:1305)
            c += 1
            w, _, u = self.q.items.pop(0)               # rwiStack.poll()
            if not skip:
                return (u, w)
            host = u[6:12]                              # hosthash (:1318)
            m = self.dd.get(host)
            if m is None:                               # first appearance: an empty queue marks the host
                self.dd[host] = ReverseQueue(MAX_RESULTS_RWI)
                return (u, w)
            m.put(w, u)                                 # second appearance (:1335,1338)
            self.dd_seq[u] = self.dd_next
            self.dd_next += 1
        if not self.dd:                                 # :1343
            return None
        # best head over all host queues (:1349-1368): the largest weight; the
        # reference breaks ties by its ConcurrentHashMap walk, here by the
        # queue order (weight, hashCode) and then the earliest queued entry
        best = None
        for host, m in self.dd.items():
            if not m.items:
                continue
            hw, hh, hu = m.items[0]
            key = (-hw, -hh, self.dd_seq[hu])
            if best is None or key < best[0]:
                best = (key, host)
        if best is None:
            return None
        m = self.dd[best[1]]
        w, _, u = m.items.pop(0)                        # m.poll() (:1377)
        if not m.items:                                 # sizeAvailable() == 0 (:1378-1383)
            del self.dd[best[1]]
        return (u, w)


def search(index: Dict[bytes, List[bytes]], include: Iterable[bytes], exclude: Iterable[bytes],
           profile: RankingProfile, language: str = "en", max_distance: int = 2147483647,
           now_ms: int = 0, k: int = 100, filt: Optional[QueryFilter] = None) -> List[Tuple[bytes, int]]:
    """End-to-end canonical RWI query: TermSearch -> normalise -> cardinal -> top-k
    (with `filt`: addRWIs constraints, and the doubledom pull order if requested)."""
    c = term_search(index, include, exclude, max_distance, now_ms)
    stack = rank(c, profile, language, now_ms, filt=filt)
    if filt is not None and filt.skip_double_dom:
        return pull_double_dom(stack, k)
    return stack[:k]
