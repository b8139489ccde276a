"""Shared helpers: load tests/golden/kats.json and run a KAT against an engine.

An engine is any object with
  term_search(index, incl, excl, max_distance, now_ms) -> (m, 40) uint8 rows
  search(index, incl, excl, profile, lang, max_distance, now_ms, k) -> [(hash, score)]
where `index` maps 12-byte term hashes to (n, 40) uint8 row arrays and
`profile` is a java_literal.RankingProfile.
"""

import json
import os

import numpy as np

import java_literal as jl

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

FIELD = {"h": (0, 12), "a": (12, 2), "s": (14, 2), "u": (16, 1), "w": (17, 2), "p": (19, 2),
         "d": (21, 1), "l": (22, 2), "x": (24, 1), "y": (25, 1), "m": (26, 1), "n": (27, 1),
         "g": (28, 1), "z": (29, 4), "c": (33, 1), "t": (34, 2), "r": (36, 1), "o": (37, 1),
         "i": (38, 1), "k": (39, 1)}


def load_kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)["kats"]


def kat_index(kat):
    return {h.encode(): np.frombuffer(b"".join(bytes.fromhex(r) for r in rows), dtype=np.uint8).reshape(-1, 40)
            for h, rows in kat["lists"].items()}


def kat_profile(kat):
    rp = jl.RankingProfile()
    spec = kat.get("profile", {})
    if spec.get("all_zero"):
        rp.all_zero()
    for k, v in spec.items():
        if k.startswith("coeff_"):
            setattr(rp, k, v)
    return rp


def field(row, name):
    off, w = FIELD[name]
    if name in ("h", "l"):
        return bytes(row[off:off + w]).decode("latin-1")
    v = 0
    for b in row[off:off + w]:
        v = (v << 8) | int(b)
    return v


def check_rows(kat, rows):
    exp = kat["expect_rows"]
    assert len(rows) == len(exp), (kat["name"], len(rows), len(exp))
    for r, e in zip(rows, exp):
        for name, v in e.items():
            assert field(r, name) == v, (kat["name"], name, field(r, name), v)


def check_hits(kat, hits):
    exp = [(h, s) for h, s in kat["expect_hits"]]
    got = [(h.decode() if isinstance(h, bytes) else h, int(s)) for h, s in hits]
    assert got == exp, (kat["name"], got, exp)


def run_kat(engine, kat):
    idx = kat_index(kat)
    incl = [h.encode() for h in kat["include"]]
    excl = [h.encode() for h in kat["exclude"]]
    if "expect_rows" in kat:
        rows = engine.term_search(idx, incl, excl, kat["max_distance"], kat["now_ms"])
        check_rows(kat, rows)
    if "expect_hits" in kat:
        hits = engine.search(idx, incl, excl, kat_profile(kat), kat.get("language", "en"),
                             kat["max_distance"], kat["now_ms"], 100)
        check_hits(kat, hits)
