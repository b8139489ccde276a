"""Shard decomposition of the canonical normalisation (TEST INFRASTRUCTURE).

Restates, in plain Python, the exchange that libyrwi performs between URL-hash
range shards (k_reduce / k_shard_fin / k_combine in yrwi_kernels.hip): every
shard summarises its part of the joined container -- min/max of the ranking
fields, its first element and its max-distance fold pieces -- and the summaries
are combined in shard (= url-hash) order.  The gloo tests check that this
composition reproduces the single-container fold of ReferenceOrder exactly
(WordReferenceVars.min/max :383-455, the distance fold :431-445).
"""

from typing import List, Tuple

import java_literal as jl

FIELDS = ["hitcount", "llocal", "lother", "wordsintext", "phrasesintext", "posintext", "posinphrase",
          "posofphrase", "urllength", "urlcomps", "wordsintitle"]


def _feat(row: bytes):
    c = lambda k: jl.col_long(row, k)  # noqa: E731
    f = {"hitcount": row[33], "llocal": row[24], "lother": row[25], "wordsintext": c("w"),
         "phrasesintext": c("p"), "posintext": c("t"), "posinphrase": row[36], "posofphrase": row[37],
         "urllength": row[26], "urlcomps": row[27], "wordsintitle": row[16]}
    tf = float(f["hitcount"]) / float(f["wordsintext"] + f["wordsintitle"] + 1)
    return f, c("a"), c("t"), row[38], tf


def shard_summary(rows: List[bytes]) -> dict:
    """Summary of one shard's (sorted) container part."""
    s = {"n": len(rows), "mn": {}, "mx": {}, "tf": None, "first": None, "va_rest": None, "segs": []}
    if not rows:
        return s
    prun = -1
    for i, r in enumerate(rows):
        f, a, p, od, tf = _feat(r)
        for k in FIELDS:
            s["mn"][k] = min(s["mn"].get(k, 1 << 30), f[k])
            s["mx"][k] = max(s["mx"].get(k, -1), f[k])
        s["tf"] = (tf, tf) if s["tf"] is None else (min(s["tf"][0], tf), max(s["tf"][1], tf))
        if i == 0:
            s["first"] = (p, od, a)
            continue
        s["va_rest"] = (a, a) if s["va_rest"] is None else (min(s["va_rest"][0], a), max(s["va_rest"][1], a))
        if p > prun:
            s["segs"].append([p, od, od])  # (P, max od, last positive od)
            prun = p
        else:
            seg = s["segs"][-1]
            seg[1] = max(seg[1], od)
            if od > 0:
                seg[2] = od
    return s


def combine(summaries: List[dict], now_ms: int) -> Tuple[dict, dict, Tuple[float, float], int, int, int]:
    """Combine shard summaries in shard order -> (min, max, tf, va_min, va_max, D)."""
    mn, mx, tf, vmn, vmx = {}, {}, None, 1 << 30, -1
    P, A, hasA = 0, 0, False
    first = True

    def piece(Pj, M, L):
        nonlocal P, A, hasA
        Pe = max(P, Pj)
        if Pe > 0:
            d0 = abs(Pe - A) if hasA else 0
            if M > d0:
                A, hasA = Pe + M, True
        elif L > 0:
            A, hasA = L, True
        P = Pe

    for s in summaries:
        if s["n"] == 0:
            continue
        for k in FIELDS:
            mn[k] = min(mn.get(k, 1 << 30), s["mn"][k])
            mx[k] = max(mx.get(k, -1), s["mx"][k])
        tf = s["tf"] if tf is None else (min(tf[0], s["tf"][0]), max(tf[1], s["tf"][1]))
        p0, od0, a0 = s["first"]
        af = jl.micro_date_days(jl.reverse_micro_date_days(a0, now_ms)) if first else a0
        vmn, vmx = min(vmn, af), max(vmx, af)
        if s["va_rest"]:
            vmn, vmx = min(vmn, s["va_rest"][0]), max(vmx, s["va_rest"][1])
        if first:
            P = p0
            first = False
        else:
            piece(p0, od0, od0)
        for Pj, M, L in s["segs"]:
            piece(Pj, M, L)
    D = abs(P - A) if (hasA and P > 0) else 0
    return mn, mx, tf, vmn, vmx, D


def shard_of(urlhash: bytes, world: int) -> int:
    """Distribution.verticalDHTPosition (Distribution.java:153-158): top log2(world)
    bits of the 63-bit Base64 cardinal = top bits of the first character."""
    e = world.bit_length() - 1
    return jl.AHPLA[urlhash[0]] >> (6 - e) if e else 0
