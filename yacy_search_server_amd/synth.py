"""Deterministic synthetic RWI index generator (ctypes front end of csrc/synth.cpp).

Builds the posting lists the way YaCy stores them: for every term a sorted run
of 40-byte ``WordReferenceRow`` rows (WordReferenceRow.java:49-72).  The
configurations C1..C5 of BASELINE.md/SURVEY.md §8(d) are named presets.
"""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))


class _Cfg(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("n_urls", ctypes.c_int64),
        ("n_terms", ctypes.c_int32),
        ("n_hosts", ctypes.c_int32),
        ("n_postings", ctypes.c_int64),
        ("zipf_df", ctypes.c_double),
        ("zipf_host", ctypes.c_double),
        ("df_clip", ctypes.c_int64),
        ("chunk_lo", ctypes.c_int32),
        ("chunk_hi", ctypes.c_int32),
    ]


_lib = None


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "libyrwi_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() first")
        lib = ctypes.CDLL(path)
        lib.yrwi_synth_df.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_void_p]
        lib.yrwi_synth_term_hash.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_int32, ctypes.c_void_p]
        lib.yrwi_synth_counts.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_int32, ctypes.c_void_p]
        lib.yrwi_synth_fill.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        lib.yrwi_synth_fill_terms.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_void_p, ctypes.c_int32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        lib.yrwi_synth_queries.argtypes =[ctypes.POINTER(_Cfg), ctypes.c_uint64, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib = lib
    return _lib


SEED_BASE = 0x5941437900000000  # seed = 0x5941437900000000 + config id


@dataclass
class SynthConfig:
    seed: int
    n_urls: int
    n_terms: int
    n_hosts: int
    n_postings: int
    zipf_df: float = 0.8
    zipf_host: float = 1.1
    df_clip: int = 50_000_000
    chunk_lo: int = 0
    chunk_hi: int = 64

    def _c(self) -> _Cfg:
        return _Cfg(self.seed, self.n_urls, self.n_terms, self.n_hosts, self.n_postings,
                    self.zipf_df, self.zipf_host, self.df_clip, self.chunk_lo, self.chunk_hi)

    def shard(self, rank: int, world: int) -> "SynthConfig":
        """URL-hash-range shard (Distribution.verticalDHTPosition, e = log2(world)):
        chunk = index of url-hash char 0; rank r owns chunks [64r/world, 64(r+1)/world)."""
        assert world & (world - 1) == 0 and world <= 64
        step = 64 // world
        return SynthConfig(self.seed, self.n_urls, self.n_terms, self.n_hosts, self.n_postings,
                           self.zipf_df, self.zipf_host, self.df_clip, rank * step, (rank + 1) * step)


PRESETS = {
    # id: (U, V, P, hosts)
    "dense": (64 * 100, 60, 120_000, 300),
    "tiny": (64 * 2000, 200, 60_000, 2_000),
    "small": (64 * 20_000, 2_000, 1_000_000, 10_000),
    "C1": (1_000_000, 10_000, 10_000_000, 50_000),
    "C2": (10_000_000, 10_000, 100_000_000, 500_000),
    "C3": (100_000_000, 10_000, 1_000_000_000, 5_000_000),
    "C5": (500_000_000, 100_000, 5_000_000_000, 5_000_000),
}


def preset(name: str, seed: Optional[int] = None) -> SynthConfig:
    U, V, P, H = PRESETS[name]
    cid = {"C1": 1, "C2": 2, "C3": 3, "C5": 5}.get(name, 0x100 + len(name))
    return SynthConfig(seed if seed is not None else SEED_BASE + cid, U, V, H, P)


def dfs(cfg: SynthConfig) -> np.ndarray:
    lib = _load()
    out = np.zeros(cfg.n_terms, dtype=np.int64)
    c = cfg._c()
    lib.yrwi_synth_df(ctypes.byref(c), out.ctypes.data)
    return out


def term_hash(cfg: SynthConfig, t: int) -> bytes:
    lib = _load()
    buf = (ctypes.c_uint8 * 12)()
    c = cfg._c()
    lib.yrwi_synth_term_hash(ctypes.byref(c), int(t), buf)
    return bytes(buf)


def counts(cfg: SynthConfig, nthreads: int = 0) -> np.ndarray:
    lib = _load()
    out = np.zeros(cfg.n_terms, dtype=np.int64)
    c = cfg._c()
    lib.yrwi_synth_counts(ctypes.byref(c), nthreads or min(16, os.cpu_count() or 1), out.ctypes.data)
    return out


@dataclass
class Index:
    """All posting lists of one (shard of a) synthetic index, concatenated.

    rows[offsets[t]:offsets[t]+sizes[t]] are term t's sorted 40-byte rows."""
    cfg: SynthConfig
    rows: np.ndarray        # (P, 40) uint8
    offsets: np.ndarray     # (V,) int64 row offsets
    sizes: np.ndarray       # (V,) int64
    hashes: List[bytes]     # term hashes

    def list_rows(self, t: int) -> np.ndarray:
        o, n = int(self.offsets[t]), int(self.sizes[t])
        return self.rows[o:o + n]

    def as_dict(self) -> Dict[bytes, np.ndarray]:
        return {self.hashes[t]: self.list_rows(t) for t in range(len(self.hashes)) if self.sizes[t] > 0}


def build_index(cfg: SynthConfig, terms: Optional[np.ndarray] = None, nthreads: int = 0) -> Index:
    """Generate the lists of `terms` (default: all terms)."""
    lib = _load()
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    sizes_all = counts(cfg, nthreads)
    if terms is None:
        terms = np.arange(cfg.n_terms)
    sizes = np.zeros(cfg.n_terms, dtype=np.int64)
    sizes[terms] = sizes_all[terms]
    offsets = np.zeros(cfg.n_terms, dtype=np.int64)
    offsets[1:] = np.cumsum(sizes)[:-1]
    total = int(sizes.sum())
    rows = np.zeros((max(total, 1), 40), dtype=np.uint8)
    c = cfg._c()
    if len(terms) == cfg.n_terms:
        lib.yrwi_synth_fill(ctypes.byref(c), 0, cfg.n_terms, offsets.ctypes.data, rows.ctypes.data, nthreads)
    else:
        tl = np.ascontiguousarray(terms, dtype=np.int32)
        offs = np.ascontiguousarray(offsets[tl], dtype=np.int64)
        lib.yrwi_synth_fill_terms(ctypes.byref(c), tl.ctypes.data, len(tl), offs.ctypes.data,
                                  rows.ctypes.data, nthreads)
    hashes = [term_hash(cfg, t) for t in range(cfg.n_terms)]
    return Index(cfg, rows[:total], offsets, sizes, hashes)


def queries(cfg: SynthConfig, nq: int, min_incl: int = 2, max_incl: int = 2, n_excl: int = 0,
            qseed: Optional[int] = None) -> List[Tuple[List[int], List[int]]]:
    """Query stream with terms sampled proportionally to df."""
    lib = _load()
    width = max_incl + n_excl
    terms = np.zeros(nq * width, dtype=np.int32)
    ni = np.zeros(nq, dtype=np.int32)
    ne = np.zeros(nq, dtype=np.int32)
    c = cfg._c()
    lib.yrwi_synth_queries(ctypes.byref(c), qseed if qseed is not None else cfg.seed ^ 0x51,
                           nq, min_incl, max_incl, n_excl, terms.ctypes.data, ni.ctypes.data,
                           ne.ctypes.data)
    out = []
    for q in range(nq):
        row = terms[q * width:(q + 1) * width]
        out.append(([int(x) for x in row[:ni[q]]], [int(x) for x in row[max_incl:max_incl + ne[q]]]))
    return out
