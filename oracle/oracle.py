"""ctypes front end of the C++ oracle (TEST INFRASTRUCTURE -- see oracle/README.md).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It loads oracle/liboracle.so (built by oracle/Makefile)."""

from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

PROFILE_ORDER = [
    "coeff_domlength", "coeff_date", "coeff_wordsintitle", "coeff_wordsintext",
    "coeff_phrasesintext", "coeff_llocal", "coeff_lother", "coeff_urllength", "coeff_urlcomps",
    "coeff_hitcount", "coeff_posintext", "coeff_posofphrase", "coeff_posinphrase",
    "coeff_authority", "coeff_worddistance", "coeff_appurl", "coeff_app_dc_title",
    "coeff_app_dc_creator", "coeff_app_dc_subject", "coeff_app_dc_description", "coeff_appemph",
    "coeff_catindexof", "coeff_cathasimage", "coeff_cathasaudio", "coeff_cathasvideo",
    "coeff_cathasapp", "coeff_urlcompintoplist", "coeff_descrcompintoplist", "coeff_prefer",
    "coeff_termfrequency", "coeff_language", "coeff_citation",
]


class YoProfile(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in PROFILE_ORDER]


class YoHit(ctypes.Structure):
    _fields_ = [("urlhash", ctypes.c_uint8 * 12), ("tiebreak", ctypes.c_int32), ("score", ctypes.c_int64)]


class YoList(ctypes.Structure):
    _fields_ = [("term", ctypes.c_void_p), ("rows", ctypes.c_void_p), ("n", ctypes.c_int64)]


class YoNorm(ctypes.Structure):
    _fields_ = [("min_f", ctypes.c_int32 * 13), ("max_f", ctypes.c_int32 * 13),
                ("min_tf", ctypes.c_double), ("max_tf", ctypes.c_double),
                ("max_distance_D", ctypes.c_int32), ("maxdomcount", ctypes.c_int32),
                ("m", ctypes.c_int64)]


class YoTrace(ctypes.Structure):
    _fields_ = [("nsteps", ctypes.c_int32), ("by_test", ctypes.c_int32 * 3),
                ("n1", ctypes.c_int64 * 3), ("n2", ctypes.c_int64 * 3), ("nout", ctypes.c_int64 * 3)]


_lib = None


def load():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
        lib = ctypes.CDLL(path)
        lib.yo_term_search.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]
        lib.yo_normalize_score.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(YoProfile),
                                           ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
        lib.yo_topk.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]
        lib.yo_search.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_int32, ctypes.POINTER(YoProfile), ctypes.c_char_p,
                                  ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                  ctypes.POINTER(ctypes.c_int32), ctypes.c_void_p, ctypes.c_void_p]
        lib.yo_join_dispatch.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32)]
        lib.yo_fold_order.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        lib.yo_profile_default.argtypes = [ctypes.POINTER(YoProfile)]
        lib.yo_join_step.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        _lib = lib
    return _lib


def default_profile() -> YoProfile:
    p = YoProfile()
    load().yo_profile_default(ctypes.byref(p))
    return p


def profile_from(obj) -> YoProfile:
    """From any object with coeff_* attributes (e.g. java_literal.RankingProfile)."""
    p = YoProfile()
    for n in PROFILE_ORDER:
        setattr(p, n, int(getattr(obj, n)))
    return p


def _lists(pairs: Sequence[Tuple[bytes, Optional[np.ndarray]]]):
    arr = (YoList * max(1, len(pairs)))()
    keep = []
    for i, (h, rows) in enumerate(pairs):
        hb = ctypes.create_string_buffer(bytes(h), 12)
        keep.append(hb)
        arr[i].term = ctypes.cast(hb, ctypes.c_void_p)
        if rows is None or len(rows) == 0:
            arr[i].rows = None
            arr[i].n = 0
        else:
            r = np.ascontiguousarray(rows, dtype=np.uint8)
            keep.append(r)
            arr[i].rows = r.ctypes.data
            arr[i].n = len(r)
    return arr, keep


def term_search(index: Dict[bytes, np.ndarray], incl: Sequence[bytes], excl: Sequence[bytes],
                max_distance: int = 2147483647, now_ms: int = 0, with_trace: bool = False):
    lib = load()
    ip, k1 = _lists([(h, index.get(h)) for h in incl])
    ep, k2 = _lists([(h, index.get(h)) for h in excl])
    cap = max([len(index.get(h, ())) for h in incl] + [1])
    out = np.zeros((cap, 40), dtype=np.uint8)
    m = ctypes.c_int64(0)
    tr = YoTrace()
    rc = lib.yo_term_search(ip, len(incl), ep, len(excl), max_distance, now_ms, out.ctypes.data, cap,
                            ctypes.byref(m), ctypes.addressof(tr))
    if rc != 0:
        raise RuntimeError(f"yo_term_search rc={rc}")
    res = out[:m.value].copy()
    return (res, tr) if with_trace else res


def normalize_score(rows: np.ndarray, profile: YoProfile, lang: str = "en", now_ms: int = 0):
    lib = load()
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    sc = np.zeros(len(rows), dtype=np.int64)
    nm = YoNorm()
    rc = lib.yo_normalize_score(rows.ctypes.data, len(rows), ctypes.byref(profile), lang.encode(),
                                now_ms, sc.ctypes.data, ctypes.addressof(nm))
    if rc != 0:
        raise RuntimeError(f"yo_normalize_score rc={rc}")
    return sc, nm


def topk(rows: np.ndarray, scores: np.ndarray, k: int, maxsize: int = 3000) -> List[Tuple[bytes, int, int]]:
    lib = load()
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    scores = np.ascontiguousarray(scores, dtype=np.int64)
    out = (YoHit * max(1, k))()
    n = ctypes.c_int32(0)
    lib.yo_topk(rows.ctypes.data, len(rows), scores.ctypes.data, maxsize, k, out, ctypes.byref(n))
    return [(bytes(out[i].urlhash), int(out[i].score), int(out[i].tiebreak)) for i in range(n.value)]


def search(index: Dict[bytes, np.ndarray], incl: Sequence[bytes], excl: Sequence[bytes] = (),
           profile: Optional[YoProfile] = None, lang: str = "en", max_distance: int = 2147483647,
           now_ms: int = 0, k: int = 100, with_norm: bool = False):
    """Canonical query; returns [(urlhash, score, tiebreak)] best first."""
    lib = load()
    profile = profile or default_profile()
    ip, k1 = _lists([(h, index.get(h)) for h in incl])
    ep, k2 = _lists([(h, index.get(h)) for h in excl])
    out = (YoHit * max(1, k))()
    n = ctypes.c_int32(0)
    nm = YoNorm()
    rc = lib.yo_search(ip, len(incl), ep, len(excl), max_distance, ctypes.byref(profile), lang.encode(),
                       now_ms, k, out, ctypes.byref(n), ctypes.addressof(nm), None)
    if rc != 0:
        raise RuntimeError(f"yo_search rc={rc}")
    hits = [(bytes(out[i].urlhash), int(out[i].score), int(out[i].tiebreak)) for i in range(n.value)]
    return (hits, nm) if with_norm else hits


def join_dispatch(n1: int, n2: int) -> Tuple[bool, bool]:
    s = ctypes.c_int32(0)
    bt = load().yo_join_dispatch(n1, n2, ctypes.byref(s))
    return bool(bt), bool(s.value)


def join_step(r1: np.ndarray, r2: np.ndarray, mode: int, max_distance: int = 2147483647,
              now_ms: int = 0) -> np.ndarray:
    """One joinConstructive step with a forced dispatch (0 enumeration, 1 by test
    small=r1, 2 by test small=r2); see yo_join_step."""
    lib = load()
    a = np.ascontiguousarray(r1, dtype=np.uint8).reshape(-1, 40)
    b = np.ascontiguousarray(r2, dtype=np.uint8).reshape(-1, 40)
    cap = max(1, min(len(a), len(b)))
    out = np.zeros((cap, 40), dtype=np.uint8)
    m = ctypes.c_int64(0)
    rc = lib.yo_join_step(a.ctypes.data if len(a) else None, len(a), b.ctypes.data if len(b) else None, len(b),
                          mode, max_distance, now_ms, out.ctypes.data, cap, ctypes.byref(m))
    if rc != 0:
        raise RuntimeError(f"yo_join_step rc={rc}")
    return out[:m.value].copy()


def fold_order(sizes: Sequence[int]) -> List[int]:
    a = np.asarray(sizes, dtype=np.int64)
    out = np.zeros(max(1, len(a)), dtype=np.int32)
    k = load().yo_fold_order(a.ctypes.data, len(a), out.ctypes.data)
    return [int(x) for x in out[:k]]
