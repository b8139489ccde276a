"""ctypes binding of libyrwi.so (the C ABI in include/yrwi.h).

The library is the only compute path: if it is missing, or no GPU is visible
when a context is opened, calls fail loudly -- there is no CPU fallback."""

from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YRWI_LIB") or os.path.join(_HERE, "libyrwi.so")  # YRWI_LIB: kernel-variant builds

PROFILE_FIELDS = [
    "coeff_domlength", "coeff_date", "coeff_wordsintitle", "coeff_wordsintext",
    "coeff_phrasesintext", "coeff_llocal", "coeff_lother", "coeff_urllength", "coeff_urlcomps",
    "coeff_hitcount", "coeff_posintext", "coeff_posofphrase", "coeff_posinphrase",
    "coeff_authority", "coeff_worddistance", "coeff_appurl", "coeff_app_dc_title",
    "coeff_app_dc_creator", "coeff_app_dc_subject", "coeff_app_dc_description", "coeff_appemph",
    "coeff_catindexof", "coeff_cathasimage", "coeff_cathasaudio", "coeff_cathasvideo",
    "coeff_cathasapp", "coeff_urlcompintoplist", "coeff_descrcompintoplist", "coeff_prefer",
    "coeff_termfrequency", "coeff_language", "coeff_citation",
]

ERRORS = {
    -1: "YRWI_E_ARG", -2: "YRWI_E_HASH", -3: "YRWI_E_UNSORTED", -4: "YRWI_E_HIP",
    -5: "YRWI_E_NOMEM", -6: "YRWI_E_RCCL", -7: "YRWI_E_NULL_LANGUAGE", -8: "YRWI_E_UNSUPPORTED",
    -9: "YRWI_E_LIMIT",
}


class CProfile(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in PROFILE_FIELDS]


class CHit(ctypes.Structure):
    _fields_ = [("urlhash", ctypes.c_uint8 * 12), ("tiebreak", ctypes.c_int32), ("score", ctypes.c_int64)]


class CFilter(ctypes.Structure):
    _fields_ = [("constraint", ctypes.c_uint8 * 4), ("has_constraint", ctypes.c_int32),
                ("all_of_constraint", ctypes.c_int32), ("contentdom", ctypes.c_int32),
                ("strict_contentdom", ctypes.c_int32), ("language", ctypes.c_char * 8),
                ("sitehash", ctypes.c_uint8 * 6), ("alt_sitehash", ctypes.c_uint8 * 6),
                ("has_sitehash", ctypes.c_int32), ("has_alt_sitehash", ctypes.c_int32),
                ("siteexcludes", ctypes.c_void_p), ("nsiteexcludes", ctypes.c_int32),
                ("urlhashes", ctypes.c_void_p), ("nurlhashes", ctypes.c_int32),
                ("skip_double_dom", ctypes.c_int32), ("flagcount", ctypes.POINTER(ctypes.c_int32))]


class CQuery(ctypes.Structure):
    _fields_ = [("incl", ctypes.c_void_p), ("nincl", ctypes.c_int32),
                ("excl", ctypes.c_void_p), ("nexcl", ctypes.c_int32),
                ("max_distance", ctypes.c_int32), ("k", ctypes.c_int32),
                ("profile", ctypes.POINTER(CProfile)), ("language", ctypes.c_char * 8),
                ("now_ms", ctypes.c_int64), ("filter", ctypes.POINTER(CFilter)),
                ("urlselection", ctypes.c_void_p), ("nurlselection", ctypes.c_int32)]


class CStats(ctypes.Structure):
    _fields_ = [("postings_in", ctypes.c_int64), ("joined", ctypes.c_int64), ("bytes_alg", ctypes.c_int64),
                ("bytes_join", ctypes.c_int64), ("t_join_ns", ctypes.c_int64), ("t_norm_ns", ctypes.c_int64),
                ("t_score_ns", ctypes.c_int64), ("t_total_ns", ctypes.c_int64),
                ("n_join_launches", ctypes.c_int32), ("n_enum_steps", ctypes.c_int32),
                ("n_test_steps", ctypes.c_int32), ("n_realloc", ctypes.c_int32),
                ("bytes_probe", ctypes.c_int64), ("t_probe_ns", ctypes.c_int64),
                ("bytes_compact", ctypes.c_int64), ("t_compact_ns", ctypes.c_int64),
                ("t_kernels_ns", ctypes.c_int64), ("bytes_probe_loaded", ctypes.c_int64),
                ("bytes_probe_capped", ctypes.c_int64), ("bytes_features", ctypes.c_int64),
                ("bytes_join_capped", ctypes.c_int64), ("bytes_alg_capped", ctypes.c_int64),
                ("n_probe_dispatches", ctypes.c_int64), ("t_probe_all_ns", ctypes.c_int64),
                ("n_rank_passes", ctypes.c_int64), ("t_reduce_ns", ctypes.c_int64), ("t_scorek_ns", ctypes.c_int64),
                ("bytes_reduce", ctypes.c_int64), ("bytes_score", ctypes.c_int64),
                ("n_chain_launches", ctypes.c_int64), ("t_chain_ns", ctypes.c_int64), ("bytes_chain", ctypes.c_int64)]


class CNode(ctypes.Structure):
    _fields_ = [("urlhash", ctypes.c_uint8 * 12), ("virtual_age", ctypes.c_int32), ("wordsintitle", ctypes.c_int32),
                ("wordcount", ctypes.c_int32), ("llocal", ctypes.c_int32), ("lother", ctypes.c_int32),
                ("flags", ctypes.c_uint8 * 4), ("host_count", ctypes.c_int32), ("language", ctypes.c_char * 8)]


class CArrival(ctypes.Structure):
    _fields_ = [("ev", ctypes.c_void_p), ("rows40", ctypes.c_void_p), ("n", ctypes.c_int64),
                ("local", ctypes.c_int32), ("rc", ctypes.c_int32)]


class CEventInfo(ctypes.Structure):
    _fields_ = [("flagcount", ctypes.c_int32 * 32), ("postings_in", ctypes.c_int64),
                ("admitted_local", ctypes.c_int64), ("admitted_remote", ctypes.c_int64),
                ("remote_arrivals", ctypes.c_int64), ("maxdomcount", ctypes.c_int32),
                ("max_distance", ctypes.c_int32), ("err", ctypes.c_int32), ("stack_size", ctypes.c_int32)]


class CAbstract(ctypes.Structure):
    _fields_ = [("word", ctypes.c_uint8 * 12), ("peer", ctypes.c_uint8 * 12), ("text", ctypes.c_void_p),
                ("len", ctypes.c_int64)]


class CPeerRequest(ctypes.Structure):
    _fields_ = [("peer", ctypes.c_uint8 * 12), ("words", ctypes.c_uint32), ("url_off", ctypes.c_int64),
                ("url_n", ctypes.c_int64)]


class CIndexInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("full_rebuilds", "incremental_updates", "repacks", "index_bytes",
                                              "index_bytes_used", "bitmap_lists")]


class CTransportInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("transport", "rank", "world", "rccl_ranks", "lanes", "lanes_own_comm",
                                              "device_peers", "mailbox")] + [("pci_bus_id", ctypes.c_char * 16)]


TRANSPORTS = {0: "none", 1: "rccl", 2: "host-staged", 3: "loopback"}


class CLoadStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("files", "records", "free_records", "bad_keys", "terms", "postings",
                                              "dropped_terms")]


# every symbol include/yrwi.h declares, with its ctypes signature
_VP = ctypes.c_void_p
SIGNATURES = {
    "yrwi_profile_default": (None, [ctypes.POINTER(CProfile)]),
    "yrwi_profile_all_zero": (None, [ctypes.POINTER(CProfile)]),
    "yrwi_profile_parse": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(CProfile)]),
    "yrwi_open": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_VP)]),
    "yrwi_open_shard": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                       ctypes.POINTER(_VP)]),
    "yrwi_get_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "yrwi_close": (None, [_VP]),
    "yrwi_last_error": (ctypes.c_char_p, [_VP]),
    "yrwi_shard_info": (ctypes.c_int, [_VP, ctypes.POINTER(CTransportInfo)]),
    "yrwi_put_list": (ctypes.c_int, [_VP, ctypes.c_char_p, _VP, ctypes.c_int64, ctypes.c_int]),
    "yrwi_build_url_ids": (ctypes.c_int, [_VP]),
    "yrwi_list_size": (ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "yrwi_get_list": (ctypes.c_int, [_VP, ctypes.c_char_p, _VP, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "yrwi_index_stats": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_int64)]),
    "yrwi_realloc_events": (ctypes.c_int64, []),
    "yrwi_index_info_get": (ctypes.c_int, [_VP, ctypes.POINTER(CIndexInfo)]),
    "yrwi_query": (ctypes.c_int, [_VP, ctypes.POINTER(CQuery), ctypes.POINTER(CHit),
                                  ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(CStats)]),
    "yrwi_query_batch": (ctypes.c_int, [_VP, ctypes.POINTER(CQuery), ctypes.c_int32, ctypes.c_int32,
                                        ctypes.POINTER(CHit), ctypes.POINTER(ctypes.c_int32),
                                        ctypes.POINTER(CStats)]),
    "yrwi_query_batch_submit": (ctypes.c_int, [_VP, ctypes.POINTER(CQuery), ctypes.c_int32, ctypes.c_int32,
                                               ctypes.POINTER(CHit), ctypes.POINTER(ctypes.c_int32),
                                               ctypes.POINTER(CStats), ctypes.POINTER(ctypes.c_int64)]),
    "yrwi_query_batch_wait": (ctypes.c_int, [_VP, ctypes.c_int64]),
    "yrwi_host_alloc": (ctypes.c_int, [_VP, ctypes.c_size_t, ctypes.POINTER(_VP)]),
    "yrwi_host_free": (ctypes.c_int, [_VP, _VP]),
    "yrwi_load_heaps": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int32, ctypes.c_int32,
                                       ctypes.POINTER(CLoadStats)]),
    "yrwi_score_nodes": (ctypes.c_int, [_VP, ctypes.POINTER(CNode), ctypes.c_int64, ctypes.POINTER(CProfile),
                                        ctypes.c_char_p, ctypes.c_int32, _VP]),
    "yrwi_event_open": (ctypes.c_int, [_VP, ctypes.POINTER(CProfile), ctypes.c_char_p, ctypes.c_int64,
                                       ctypes.c_int32, ctypes.POINTER(CFilter), ctypes.c_int64, _VP]),
    "yrwi_settle_scratch": (ctypes.c_int, [_VP]),
    "yrwi_event_source": (ctypes.c_int, [_VP, _VP, ctypes.c_char_p, ctypes.c_int32, _VP, _VP]),
    "yrwi_event_open_order": (ctypes.c_int, [_VP, ctypes.POINTER(CProfile), ctypes.c_char_p, ctypes.c_int64,
                                             ctypes.c_int64, _VP]),
    "yrwi_event_add": (ctypes.c_int, [_VP, ctypes.POINTER(CArrival), ctypes.c_int32]),
    "yrwi_event_result": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(CHit), ctypes.c_int32,
                                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(CEventInfo)]),
    "yrwi_check_url_ids": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "yrwi_hostx_selftest": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int32,
                                           ctypes.c_int64]),
    "yrwi_event_pull": (ctypes.c_int, [_VP, _VP, ctypes.c_int32, ctypes.POINTER(CHit), ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_int32)]),
    "yrwi_event_close": (None, [_VP, _VP]),
    "yrwi_event_order": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int64, ctypes.c_int32, _VP]),
    "yrwi_event_authority": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int32, _VP]),
    "yrwi_index_abstracts": (ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p, _VP,
                                            ctypes.c_int64, _VP, ctypes.POINTER(ctypes.c_int32)]),
    "yrwi_secondary_search": (ctypes.c_int, [_VP, ctypes.POINTER(CAbstract), ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int32, _VP, _VP,
                                             ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                             ctypes.POINTER(CPeerRequest), ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_int32), _VP, _VP,
                                             ctypes.POINTER(ctypes.c_int32)]),
    "yrwi_join_exclude": (ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int64, _VP, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_int64)]),
    "yrwi_term_search": (ctypes.c_int, [_VP, ctypes.POINTER(CQuery), _VP, ctypes.c_int64,
                                        ctypes.POINTER(ctypes.c_int64)]),
    "yrwi_normalize_score": (ctypes.c_int, [_VP, _VP, ctypes.c_int64, ctypes.POINTER(CProfile), ctypes.c_char_p,
                                            ctypes.c_int64, _VP]),
}

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class YrwiError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"{ERRORS.get(rc, rc)}: {msg}")
        self.rc = rc
