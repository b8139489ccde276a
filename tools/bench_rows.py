"""Throughput of the §8f rows beside the headline path:

* search events (row 3): E concurrent SearchEvents, each receiving remote
  containers of R rows per call (Protocol.remoteSearchProcess -> addRWIs), one
  yrwi_event_add call per round carrying one arrival for every event;
* index abstracts (row 3): compressIndex over the largest lists of the corpus;
* secondary search (row 3): decompress + join of the abstracts of P peers;
* node scoring (row 4): cardinal(URIMetadataNode) over N nodes.

Prints one JSON object.  Times are host wall clock around the C-ABI call (the
call returns when the results are in host memory)."""

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from yacy_search_server_amd import RWIIndex, synth  # noqa: E402
from yacy_search_server_amd import _lib  # noqa: E402


def bench_events(ix, pool, rng, nev, rows_per, rounds, k):
    L = _lib.lib()
    evs = [ix.event(None, "en", 20741 * 86400000, k=k, max_postings=rows_per * rounds + 16) for _ in range(nev)]
    calls = []
    keep = []
    for r in range(rounds):
        arr = (_lib.CArrival * nev)()
        for e in range(nev):
            rows = np.ascontiguousarray(pool[rng.integers(0, len(pool), rows_per)])
            keep.append(rows)
            arr[e].ev = evs[e]._e
            arr[e].rows40 = rows.ctypes.data
            arr[e].n = rows_per
            arr[e].local = 0
        calls.append(arr)
    # warm-up on separate events
    warm = [ix.event(None, "en", 20741 * 86400000, k=k, max_postings=rows_per + 16) for _ in range(nev)]
    wa = (_lib.CArrival * nev)()
    for e in range(nev):
        wa[e].ev = warm[e]._e
        wa[e].rows40 = keep[e].ctypes.data
        wa[e].n = rows_per
    assert L.yrwi_event_add(ix._h, wa, nev) == 0
    for w in warm:
        w.close()
    t0 = time.perf_counter()
    for arr in calls:
        assert L.yrwi_event_add(ix._h, arr, nev) == 0
    dt = time.perf_counter() - t0
    for e in evs:
        e.close()
    n = nev * rows_per * rounds
    return {"events": nev, "rows_per_arrival": rows_per, "rounds": rounds, "k": k,
            "postings": n, "seconds": round(dt, 4), "postings_per_s": n / dt,
            "ms_per_call": round(dt / rounds * 1e3, 3)}


def bench_abstracts(ix, idx, nterms):
    L = _lib.lib()
    order = [int(t) for t in np.argsort(-idx.sizes)[:nterms]]
    terms = b"".join(idx.hashes[t] for t in order)
    post = int(sum(idx.sizes[t] for t in order))
    cap = 14 * post + 2 * nterms
    out = ctypes.create_string_buffer(cap)
    offs = (ctypes.c_int64 * (nterms + 1))()
    nout = ctypes.c_int32()
    assert L.yrwi_index_abstracts(ix._h, terms, 1, None, out, cap, offs, ctypes.byref(nout)) == 0
    t0 = time.perf_counter()
    assert L.yrwi_index_abstracts(ix._h, terms, nterms, None, out, cap, offs, ctypes.byref(nout)) == 0
    dt = time.perf_counter() - t0
    return {"terms": nterms, "postings": post, "abstract_bytes": int(offs[nterms]), "seconds": round(dt, 4),
            "postings_per_s": post / dt}


def bench_secondary(ix, idx, npeers, rng):
    """npeers peers answer a 3-word query; peer p sends, for every word, the
    abstract of list 200+p (~50K postings): the words' maps are the union of the
    peers' lists, the join is that union, each url asked from its newest peer."""
    srt = np.argsort(-idx.sizes)
    words = [idx.hashes[int(t)] for t in srt[:3]]
    texts = ix.index_abstracts([idx.hashes[int(srt[200 + p])] for p in range(npeers)])
    abstracts = []
    for p in range(npeers):
        peer = ("peer%08d" % p).encode()
        for w in words:
            abstracts.append((w, peer, texts[p]))
    ix.secondary_search(abstracts[:3], 3, b"mypeerAAAAAA")
    t0 = time.perf_counter()
    nj, npl = ix.secondary_search(abstracts, 3, b"mypeerAAAAAA", decode=False)
    dt = time.perf_counter() - t0
    nb = sum(len(a[2]) for a in abstracts)
    return {"peers": npeers, "abstracts": len(abstracts), "abstract_bytes": nb, "joined_urls": nj,
            "requests": npl, "seconds": round(dt, 4), "abstract_MB_per_s": nb / dt / 1e6}


def bench_nodes(ix, n, rng):
    L = _lib.lib()
    nodes = np.zeros(n, dtype=np.dtype(_lib.CNode))
    alpha = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_", dtype=np.uint8)
    hs = rng.integers(0, 64, (n, 12))
    nodes["urlhash"] = alpha[hs]
    nodes["virtual_age"] = hs[:, 0] * 300
    nodes["wordcount"] = hs[:, 1] * 50
    nodes["language"][:, 0] = ord("e")
    nodes["language"][:, 1] = ord("n")
    arr = ctypes.cast(nodes.ctypes.data, ctypes.POINTER(_lib.CNode))
    out = np.zeros(n, dtype=np.int64)
    prof = _lib.CProfile()
    L.yrwi_profile_default(ctypes.byref(prof))
    L.yrwi_score_nodes(ix._h, arr, n, ctypes.byref(prof), b"en", 0, out.ctypes.data)
    t0 = time.perf_counter()
    reps = 10
    for _ in range(reps):
        assert L.yrwi_score_nodes(ix._h, arr, n, ctypes.byref(prof), b"en", 0, out.ctypes.data) == 0
    dt = (time.perf_counter() - t0) / reps
    return {"nodes": n, "seconds": round(dt, 5), "nodes_per_s": n / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--events", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=16)
    ap.add_argument("--k", type=int, default=100)
    args = ap.parse_args()
    rng = np.random.default_rng(1)
    cfg = synth.preset(args.config)
    idx = synth.build_index(cfg)
    ix = RWIIndex(0)
    for t in range(cfg.n_terms):
        if idx.sizes[t]:
            ix.add(idx.hashes[t], idx.list_rows(t))
    pool = np.asarray(idx.rows, dtype=np.uint8)
    out = {"config": args.config}
    steps = [("events", lambda: bench_events(ix, pool, rng, args.events, args.rows, args.rounds, args.k)),
             ("events_large", lambda: bench_events(ix, pool, rng, 64, 20000, 4, args.k)),
             ("index_abstracts", lambda: bench_abstracts(ix, idx, 8)),
             ("secondary_search", lambda: bench_secondary(ix, idx, 16, rng)),
             ("score_nodes", lambda: bench_nodes(ix, 1 << 18, rng))]
    for name, fn in steps:
        print("bench_rows:", name, file=sys.stderr, flush=True)
        out[name] = fn()
        print("bench_rows:", name, "done", out[name], file=sys.stderr, flush=True)
    print(json.dumps(out))
    ix.close()


if __name__ == "__main__":
    main()
