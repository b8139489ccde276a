"""Shard decomposition of the canonical normalisation (TEST INFRASTRUCTURE).

Restates, in plain Python, the exchange that libyrwi performs between URL-hash
range shards (k_reduce / k_shard_fin / k_combine in yrwi_kernels.hip): every
shard summarises its part of the joined container -- min/max of the ranking
fields, its first element and its max-distance fold pieces -- and the summaries
are combined in shard (= url-hash) order.  The gloo tests check that this
composition reproduces the single-container fold of ReferenceOrder exactly
(WordReferenceVars.min/max :383-455, the distance fold :431-445).
"""

from typing import Callable, Dict, List, Sequence, Tuple

import numpy as np

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


def _b64key(h: bytes):
    return [jl.AHPLA[c] for c in h]


def shard_term_search(local: Dict[bytes, np.ndarray], incl: Sequence[bytes], excl: Sequence[bytes],
                      max_distance: int, now_ms: int, allsum: Callable[[List[int]], List[int]]) -> np.ndarray:
    """TermSearch + joinExcludeContainers on ONE url-hash shard, the way libyrwi
    runs it (yrwi_host.cpp plan_query / run_join_phase).

    Every decision the reference takes on container sizes is taken on the GLOBAL
    sizes -- the sum over shards, obtained with ``allsum`` (element-wise sum of a
    list of ints over all ranks; every rank makes the same sequence of calls):
      J1  a missing include term empties the result, a missing exclude term
          disables exclusion (AbstractIndex.java:108-127);
      J2  the fold order (int)(size*1000 + i) (ReferenceContainer.java:334-366);
      J3  the dispatch of every step, including the size of the intermediate
          joined container (:406-416).
    The rows joined are the shard's own, so the concatenation of the shards'
    results in shard order is the single-container result."""
    import oracle as orc
    inc = sorted({bytes(h) for h in incl}, key=_b64key)
    exc = sorted({bytes(h) for h in excl}, key=_b64key)
    empty = np.zeros((0, 40), dtype=np.uint8)
    lists = {h: (local[h] if h in local else empty) for h in inc + exc}
    g = allsum([len(lists[h]) for h in inc + exc])
    gi, ge = g[:len(inc)], g[len(inc):]
    if not inc or min(gi) == 0:
        return empty
    use_excl = len(exc) > 0 and min(ge) > 0
    order = orc.fold_order(gi)
    acc, acc_g = lists[inc[order[0]]], gi[order[0]]
    for j in order[1:]:
        if acc_g == 0:
            break
        bt, small_is_1 = orc.join_dispatch(acc_g, gi[j])
        mode = (1 if small_is_1 else 2) if bt else 0
        acc = orc.join_step(acc, lists[inc[j]], mode, max_distance, now_ms)
        acc_g = allsum([len(acc)])[0]
    if acc_g == 0 or len(acc) == 0:
        return empty
    if use_excl:
        keep = np.ones(len(acc), dtype=bool)
        ak = [bytes(r[:12]) for r in acc]
        for h in exc:
            ex = {bytes(r[:12]) for r in lists[h]}
            keep &= np.array([k not in ex for k in ak], dtype=bool)
        acc = acc[keep]
    return acc


def lockstep_allsum(world: int):
    """allsum callables for `world` threads simulating the ranks in one process."""
    import threading
    bar = threading.Barrier(world)
    slots: List[List[int]] = [None] * world  # type: ignore[list-item]
    out: List[List[int]] = [None]  # type: ignore[list-item]

    def make(rank: int):
        def allsum(v: List[int]) -> List[int]:
            slots[rank] = list(v)
            if bar.wait() == 0:
                out[0] = [sum(x) for x in zip(*slots)]
            bar.wait()
            res = list(out[0])
            bar.wait()
            return res
        return allsum
    return [make(r) for r in range(world)]


def sharded_term_search(parts: List[Dict[bytes, np.ndarray]], incl, excl, max_distance: int = 2147483647,
                        now_ms: int = 0, protocol: str = "global") -> List[np.ndarray]:
    """All shards of one query in one process.  protocol "global" is libyrwi's
    (shard_term_search); "local" plans every shard on its own list sizes (the
    round-1 behaviour, kept to show what it breaks)."""
    import threading
    import oracle as orc
    W = len(parts)
    if protocol == "local":
        return [orc.term_search(p, incl, excl, max_distance, now_ms) for p in parts]
    fns = lockstep_allsum(W)
    res: List[np.ndarray] = [None] * W  # type: ignore[list-item]
    errs = []

    def run(r):
        try:
            res[r] = shard_term_search(parts[r], incl, excl, max_distance, now_ms, fns[r])
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(repr(e))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise RuntimeError(errs[0])
    return res


def shard_of(urlhash: bytes, world: int) -> int:
    """Distribution.verticalDHTPosition (Distribution.java:153-158): top log2(world)
    bits of the 63-bit Base64 cardinal = top bits of the first character."""
    e = world.bit_length() - 1
    return jl.AHPLA[urlhash[0]] >> (6 - e) if e else 0
