"""YaCy BLOB heap loader.

CPU: the restatement in oracle/heap.py against hand-derived expectations of the
cited reference lines (record scan, import rules, file and RAM precedence).
GPU: yrwi_load_heaps against oracle.heap.index_get on synthetic heap files with
overlapping terms and url hashes, then full queries over the loaded index
against the oracle.  No reference test covers the heap format (parity of the
loader rests on the restatement)."""

import os
import struct

import numpy as np
import pytest

import heap
import oracle as orc
from yacy_search_server_amd import synth

NOW = 20741 * 86400000


def _rows(hashes, tag):
    """Hand-built rows: url hash + a recognisable feature byte (hitcount) = tag."""
    out = np.zeros((len(hashes), 40), np.uint8)
    for i, h in enumerate(hashes):
        out[i, :12] = np.frombuffer(h, np.uint8)
        out[i, 22:24] = np.frombuffer(b"en", np.uint8)
        out[i, 33] = tag
    return out


H = [b"AAAAAAhost01", b"BBBBBBhost01", b"CCCCCChost02", b"DDDDDDhost02", b"EEEEEEhost03"]
T1, T2, T3 = b"termAAAAAAAA", b"termBBBBBBBB", b"termCCCCCCCC"


def test_record_scan_rules(tmp_path):
    p = str(tmp_path / "text.index.20240101000000000.blob")
    good = heap.export_collection(_rows(H[:2], 1))
    with open(p, "wb") as f:
        f.write(struct.pack(">i", 12 + len(good)) + T1 + good)                     # live record
        f.write(struct.pack(">i", 12 + 20) + b"\0" + T2[1:] + b"x" * 20)            # free record (key[0] == 0)
        f.write(struct.pack(">i", 12 + len(good)) + b"te rm!!AAAAA" + good)          # not well-formed -> skipped
        f.write(struct.pack(">i", 12 + len(good)) + T3 + good)                     # live
        f.write(struct.pack(">i", 0) + T2 + good)                                    # reclen 0: file ends here
        f.write(struct.pack(">i", 12 + len(good)) + T2 + good)
    recs = heap.scan_heap(p)
    assert sorted(recs) == [T1, T3]
    assert recs[T1] == good


def test_import_rules():
    r = _rows(H[:3], 7)
    assert len(heap.import_rowset(heap.export_collection(r))) == 3
    assert len(heap.import_rowset(b"\0" * 10)) == 0                               # shorter than the header
    assert len(heap.import_rowset(heap.export_collection(r, size=-1 & 0xFFFFFFFF))) == 0  # size < 0
    with pytest.raises(heap.SpaceExceeded):
        heap.import_rowset(heap.export_collection(r, size=4))                       # size*40 != len - 14
    # unsorted tail past orderbound is sorted, first of equal url hashes kept
    t = np.concatenate([_rows([H[0], H[3]], 1), _rows([H[1], H[0]], 2)])
    got = heap.import_rowset(heap.export_collection(t, orderbound=2))
    assert [bytes(x[:12]) for x in got] == [H[0], H[1], H[3]] and got[0, 33] == 1


def test_file_and_ram_precedence(tmp_path):
    old = str(tmp_path / "text.index.20230101000000000.blob")
    new = str(tmp_path / "text.index.20240101000000000.blob")
    heap.write_heap(old, [(T1, heap.export_collection(_rows([H[0], H[2]], 1)))])
    heap.write_heap(new, [(T1, heap.export_collection(_rows([H[0], H[1], H[4]], 2))),
                          (T2, heap.export_collection(_rows([H[3]], 2)))])
    ram = {T1: _rows([H[1], H[3]], 3), T3: _rows([H[4]], 3)}
    files = heap.order_files([new, old, str(tmp_path / "unstamped.blob")])
    assert files == [old, new]
    got = heap.index_get(files, ram)
    t1 = got[T1]
    assert [bytes(x[:12]) for x in t1] == [H[0], H[1], H[2], H[3], H[4]]
    # H0: old file wins over new; H1: file wins over RAM; H3: RAM only
    assert list(t1[:, 33]) == [1, 2, 1, 3, 2]
    assert list(got[T3][:, 33]) == [3] and list(got[T2][:, 33]) == [2]


def test_spaceexceeded_drops_blob_part(tmp_path):
    p = str(tmp_path / "text.index.20240101000000000.blob")
    heap.write_heap(p, [(T1, heap.export_collection(_rows(H[:2], 1), size=3))])
    got = heap.index_get([p], {T1: _rows([H[4]], 3)})
    assert [bytes(x[:12]) for x in got[T1]] == [H[4]]


# ------------------------------------------------------------------- GPU
def _synth_heaps(tmp_path, cfg, idx, nfiles=3, seed=5):
    """Split every list over nfiles heap files with overlaps and modified features,
    so that the file order decides which row survives."""
    rng = np.random.default_rng(seed)
    paths = []
    recs = [[] for _ in range(nfiles)]
    ram = {}
    for t in range(cfg.n_terms):
        rows = idx.list_rows(t)
        if len(rows) == 0:
            continue
        for f in range(nfiles):
            m = rng.random(len(rows)) < 0.5
            if m.any():
                r = rows[m].copy()
                r[:, 33] = (r[:, 33].astype(int) + f + 1) % 256  # hitcount tells the files apart
                recs[f].append((idx.hashes[t], heap.export_collection(r)))
        if t % 3 == 0:
            m = rng.random(len(rows)) < 0.3
            if m.any():
                ram[idx.hashes[t]] = rows[m].copy()
    for f in range(nfiles):
        rng.shuffle(recs[f])
        p = str(tmp_path / f"text.index.2024010100000{f}000.blob")
        heap.write_heap(p, recs[f])
        paths.append(p)
    return paths, ram


@pytest.mark.gpu
def test_load_heaps_gpu_matches_oracle(tmp_path):
    from yacy_search_server_amd import Query, RWIIndex
    cfg = synth.preset("tiny")
    idx = synth.build_index(cfg)
    paths, ram = _synth_heaps(tmp_path, cfg, idx)
    ix = RWIIndex(0)
    try:
        for h, r in ram.items():
            ix.add(h, r)
        st = ix.load_heaps(list(reversed(paths)), order_by_name=True)
        exp = heap.index_get(heap.order_files(paths), ram)
        assert st.files == len(paths) and st.dropped_terms == 0
        assert st.terms == len(exp) and st.postings == sum(len(v) for v in exp.values())
        for h, rows in exp.items():
            assert ix.get_size(h) == len(rows)
            got = ix.term_search([h], now_ms=NOW)
            assert np.array_equal(got, rows), h
        qs = synth.queries(cfg, 12, 1, 3, 1, qseed=77)
        for inc, exc in qs:
            q = Query([idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], now_ms=NOW)
            g = ix.search(q.include, q.exclude, now_ms=NOW, k=100)
            e = orc.search(exp, q.include, q.exclude, now_ms=NOW, k=100)
            assert [(x.urlhash, x.score) for x in g] == [(a, b) for a, b, _ in e]
    finally:
        ix.close()


@pytest.mark.gpu
def test_load_heaps_gpu_edge_records(tmp_path):
    from yacy_search_server_amd import RWIIndex
    p = str(tmp_path / "text.index.20240101000000000.blob")
    good = heap.export_collection(_rows(H[:3], 1))
    with open(p, "wb") as f:
        f.write(struct.pack(">i", 12 + len(good)) + T1 + good)
        f.write(struct.pack(">i", 12 + 20) + b"\0" + T2[1:] + b"x" * 20)
        bad = heap.export_collection(_rows(H[:2], 1), size=5)
        f.write(struct.pack(">i", 12 + len(bad)) + T2 + bad)
        f.write(struct.pack(">i", 12 + len(good)) + b"te rm!!AAAAA" + good)
        f.write(struct.pack(">i", 0) + T3 + good)
    ix = RWIIndex(0)
    try:
        ix.add(T2, _rows([H[4]], 3))
        st = ix.load_heaps([p])
        assert (st.records, st.free_records, st.bad_keys, st.dropped_terms, st.terms) == (2, 1, 1, 1, 1)
        assert np.array_equal(ix.term_search([T1], now_ms=NOW), _rows(H[:3], 1))
        assert np.array_equal(ix.term_search([T2], now_ms=NOW), _rows([H[4]], 3))  # RAM part kept
        assert ix.get_size(T3) == 0
    finally:
        ix.close()
