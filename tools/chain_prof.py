"""k_chain path counters for one C3 batch (profiling build: YRWI_LIB=.../libyrwi_cprof.so,
built with EXTRA=-DYRWI_CHAIN_PROF).  Prints which search path every (group, list) of the
chained step took and the matches behind it, and the cycles spent."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from yacy_search_server_amd import RWIIndex, RankingProfile, Query, synth, _lib  # noqa: E402

NAMES = ["groups", "matches", "bm_tests", "bm_lists", "lds_tests", "lds_lists", "h1_tests", "h1_lists",
         "h2_tests", "h2_lists", "key_tests", "key_lists", "tiles", "rounds", "search_cycles", "wg_cycles",
         "survivors", "", "", "", "", "", "", ""]


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "C3"
    nincl = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    nexcl = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    cfg = synth.preset(preset)
    if len(sys.argv) > 5:  # url-hash shard r of n (C5: shard 0 of 8)
        cfg = cfg.shard(0, int(sys.argv[5]))
    idx = synth.build_index(cfg)
    ix = RWIIndex(0)
    for t in range(cfg.n_terms):
        if idx.sizes[t]:
            ix.add(idx.hashes[t], idx.list_rows(t))
    ix.build_url_ids()
    hashes = [synth.term_hash(cfg, t) for t in range(cfg.n_terms)]
    maxi = int(os.environ.get("CP_MAX_TERMS", nincl))
    qs = synth.queries(synth.preset(preset), 1000, nincl, maxi, nexcl)
    prof = RankingProfile()
    if len(sys.argv) > 4 and sys.argv[4] == "custom":
        prof.coeff_date, prof.coeff_domlength, prof.coeff_authority, prof.coeff_termfrequency = 15, 15, 13, 10
    batch = [Query([hashes[t] for t in inc], [hashes[t] for t in exc], k=100, profile=prof) for inc, exc in qs]
    f = _lib.lib().yrwi_chain_prof
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    out = (ctypes.c_ulonglong * 24)()
    ix.search_batch(batch)  # warm-up
    f(out)
    res = []
    for _ in range(3):
        t0 = time.time()
        ix.search_batch(batch)
        dt = time.time() - t0
        f(out)
        res.append({**{n: int(out[i]) for i, n in enumerate(NAMES) if n}, "wall_ms": round(dt * 1e3, 2)})
    print(json.dumps(res[-1]))
    ix.close()


if __name__ == "__main__":
    main()
