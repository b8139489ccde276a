"""YaCy BLOB heap files of the reverse word index (TEST INFRASTRUCTURE -- see oracle/README.md).

Restatement of the on-disk side of IndexCell.get (paths relative to
/root/reference/source/net/yacy), used as the checker of libyrwi's loader
(yrwi_load_heaps) and to write fixture files for it:

  record layout     kelondro/blob/HeapWriter.java:57-63,114-124
                    [int32 BE reclen][key: keylength bytes][blob: reclen - keylength bytes]
  heap scan         kelondro/blob/HeapReader.java:250-304
                    reclen == 0 ends the file (the rest is cut off); a short read
                    ends it too; key[0] == 0 is a free record; a key that is not
                    well-formed Base64 is skipped; a key seen again replaces the
                    earlier record (RowHandleMap put)
  blob = export     kelondro/index/RowCollection.java:175-231 (exportRow: size-4,
                    lastread-2, lastwrote-2, orderkey-2, orderbound-4, rows)
  import            kelondro/index/RowSet.java:81-109 (importRowSet): size < 0 or
                    orderbound < 0 -> empty set; size * 40 != len - 14 ->
                    SpaceExceededException
  file order        kelondro/blob/ArrayStack.java:182-229: files named
                    <prefix>.<yyyyMMddHHmmssSSS>.blob, opened oldest first
  multi-file merge  kelondro/rwi/ReferenceContainerArray.java:305-322 (fold over the
                    files in that order) with RowSet.mergeEnum (RowSet.java:506-559):
                    on equal url hashes the row of the accumulated (older) side wins
  RAM u BLOB        kelondro/rwi/IndexCell.java:353-386: result = blobs.merge(ram),
                    the BLOB row wins; a SpaceExceededException while reading the
                    BLOBs drops the BLOB part of that term (:357-360)

Deterministic choices where the reference is not (parity unpinned, no reference
test covers the heap format): rows past orderbound are sorted stably (the
reference's quicksort, cora/sorting/Array.java:99-170, is not stable) and only
the first row of equal url hashes is kept.
"""

from __future__ import annotations

import re
import struct
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

KEYLEN = 12
ROW = 40
EXPORT_OVERHEAD = 14  # RowCollection.exportOverheadSize (:174)
ALPHA = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
_AHP = {c: i for i, c in enumerate(ALPHA)}
_STAMP = re.compile(r"\.(\d{17})\.blob$")


class SpaceExceeded(Exception):
    pass


def wellformed(key: bytes) -> bool:
    """Base64Order.wellformed (Base64Order.java:96-106): every byte in the alphabet."""
    return all(c in _AHP for c in key)


def key_order(h: bytes) -> Tuple[int, ...]:
    return tuple(_AHP[c] for c in h)


# ------------------------------------------------------------------ writing
def export_collection(rows: np.ndarray, lastread: int = 0, lastwrote: int = 0, orderkey: bytes = b"__",
                      orderbound: Optional[int] = None, size: Optional[int] = None) -> bytes:
    """RowCollection.exportCollection (:209-224): the 14-byte export header + rows.
    orderbound/size default to len(rows) (exportCollection sorts first)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, ROW)
    n = len(rows) if size is None else size
    ob = len(rows) if orderbound is None else orderbound
    hdr = struct.pack(">I", n & 0xFFFFFFFF) + struct.pack(">H", lastread & 0xFFFF) + \
        struct.pack(">H", lastwrote & 0xFFFF) + orderkey[:2].ljust(2, b"_") + struct.pack(">I", ob & 0xFFFFFFFF)
    return hdr + rows.tobytes()


def write_heap(path: str, records: Iterable[Tuple[bytes, bytes]]) -> None:
    """HeapWriter.add (:114-124) for each (key, blob), in order."""
    with open(path, "wb") as f:
        for key, blob in records:
            key = (key + b"\0" * KEYLEN)[:KEYLEN]  # HeapReader.normalizeKey (:147-157)
            f.write(struct.pack(">i", KEYLEN + len(blob)))
            f.write(key)
            f.write(blob)


# ------------------------------------------------------------------ reading
def scan_heap(path: str) -> Dict[bytes, bytes]:
    """HeapReader.initIndexReadFromHeap (:250-304) + get: key -> blob."""
    data = open(path, "rb").read()
    out: Dict[bytes, bytes] = {}
    seek = 0
    while True:
        if seek + 4 + KEYLEN > len(data):
            break  # EOF while reading the length or the key
        reclen = struct.unpack_from(">i", data, seek)[0]
        if reclen == 0:
            break  # "very bad file inconsistency": the file is cut here
        key = data[seek + 4:seek + 4 + KEYLEN]
        if key[0] != 0 and wellformed(key):
            end = seek + 4 + reclen
            if reclen >= KEYLEN and end <= len(data):
                out[key] = data[seek + 4 + KEYLEN:end]
        if reclen < 0:
            break
        seek += 4 + reclen
    return out


def import_rowset(blob: bytes) -> np.ndarray:
    """RowSet.importRowSet (:81-109) followed by RowCollection.sort (:684-692)."""
    if len(blob) < EXPORT_OVERHEAD:
        return np.zeros((0, ROW), np.uint8)
    size = struct.unpack_from(">i", blob, 0)[0]
    if size < 0:
        return np.zeros((0, ROW), np.uint8)
    orderbound = struct.unpack_from(">i", blob, 10)[0]
    if orderbound < 0:
        return np.zeros((0, ROW), np.uint8)
    if size * ROW != len(blob) - EXPORT_OVERHEAD:
        raise SpaceExceeded("importRowSet: alloc != b.length - exportOverheadSize")
    rows = np.frombuffer(blob, np.uint8, size * ROW, EXPORT_OVERHEAD).reshape(-1, ROW)
    return sort_unique(rows)


_LUT = np.full(256, -1, np.int64)
for _i, _c in enumerate(ALPHA):
    _LUT[_c] = _i


def _keys(rows: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """72-bit Base64Order key (alphabet index per char, Base64Order.java:533-553) as
    (chars 0-5, chars 6-11), each a 36-bit integer: lexicographic = key order."""
    c = _LUT[rows[:, :12]]
    w = np.array([1 << (6 * (5 - i)) for i in range(6)], np.int64)
    return c[:, :6] @ w, c[:, 6:] @ w


def sort_unique(rows: np.ndarray) -> np.ndarray:
    """Stable sort by url hash; the first of equal url hashes is kept."""
    if len(rows) == 0:
        return rows.copy()
    k0, k1 = _keys(rows)
    order = np.lexsort((np.arange(len(rows)), k1, k0))
    k0, k1 = k0[order], k1[order]
    keep = np.ones(len(rows), bool)
    keep[1:] = (k0[1:] != k0[:-1]) | (k1[1:] != k1[:-1])
    return rows[order[keep]].copy()


def merge_enum(c0: np.ndarray, c1: np.ndarray) -> np.ndarray:
    """RowSet.mergeEnum (:506-559): union of two sorted sets, c0's row on equal keys."""
    return sort_unique(np.concatenate([c0.reshape(-1, ROW), c1.reshape(-1, ROW)]))


def order_files(paths: Sequence[str]) -> List[str]:
    """ArrayStack (:182-229): files with a 17-digit stamp, oldest first."""
    stamped = [(m.group(1), p) for p in paths for m in [_STAMP.search(p)] if m]
    return [p for _, p in sorted(stamped)]


def index_get(paths: Sequence[str], ram: Optional[Dict[bytes, np.ndarray]] = None,
              shard: Tuple[int, int] = (0, 1)) -> Dict[bytes, np.ndarray]:
    """IndexCell.get for every term: BLOB files (already in ArrayStack order) folded
    with mergeEnum, then merged with the RAM container; optionally restricted to one
    url-hash shard (Distribution.verticalDHTPosition, Distribution.java:153-158)."""
    scans = [scan_heap(p) for p in paths]
    terms = set()
    for s in scans:
        terms.update(s)
    ram = ram or {}
    terms.update(ram)
    rank, world = shard
    bits = world.bit_length() - 1
    out: Dict[bytes, np.ndarray] = {}
    for t in sorted(terms):
        blob_part = None
        try:
            for s in scans:
                if t in s:
                    c = import_rowset(s[t])
                    blob_part = c if blob_part is None else merge_enum(blob_part, c)
        except SpaceExceeded:
            blob_part = None  # IndexCell.get :357-360
        r = ram.get(t)
        if r is not None:
            r = sort_unique(np.ascontiguousarray(r, np.uint8).reshape(-1, ROW))
        if blob_part is not None and r is not None:
            res = merge_enum(blob_part, r)
        else:
            res = blob_part if blob_part is not None else r
        if res is None:
            continue
        if world > 1 and len(res):
            res = res[(_LUT[res[:, 0]] >> (6 - bits)) == rank]
        if len(res):
            out[t] = res
    return out
