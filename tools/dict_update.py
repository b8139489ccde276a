"""Time url-dictionary maintenance on the C2 index (one GPU): the first full
build, then incremental updates -- a list whose urls all exist, a list of fresh
urls, a replaced list -- each followed by the consistency check, and a forced
full rebuild for comparison.  One JSON line to stdout."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from yacy_search_server_amd import RWIIndex, synth  # noqa: E402


def timed(f):
    t0 = time.perf_counter()
    f()
    return round((time.perf_counter() - t0) * 1e3, 2)


def main():
    cfg = synth.preset(os.environ.get("DICT_CONFIG", "C2"))
    idx = synth.build_index(cfg)
    ix = RWIIndex(0)
    for t in range(cfg.n_terms):
        if idx.sizes[t]:
            ix.add(idx.hashes[t], idx.list_rows(t))
    out = {"config": cfg.name if hasattr(cfg, "name") else "C2", "postings": int(idx.sizes.sum())}
    out["full_build_ms"] = timed(ix.build_url_ids)
    out["nurls"] = ix.check_url_ids()[1]
    big = int(np.argmax(idx.sizes))
    rows = idx.list_rows(big)
    # 1: a new term over existing urls (no id moves)
    ix.add(b"DICTupdate01", rows[::4].copy())
    out["add_existing_urls_ms"] = timed(ix.build_url_ids)
    out["add_existing_n"] = int(len(rows[::4]))
    # 2: a new term with fresh url hashes (every id after them moves)
    fresh = rows[: 200_000].copy()
    fresh[:, 0] = ord("_")  # url hashes beyond every synthetic one (Base64Order: '_' is last)
    ix.add(b"DICTupdate02", fresh, sorted=False)
    out["add_fresh_urls_ms"] = timed(ix.build_url_ids)
    out["add_fresh_n"] = int(len(fresh))
    fresh2 = rows[200_000: 400_000].copy()
    fresh2[:, 0] = ord("A")  # url hashes before most ids: the whole dictionary shifts
    ix.add(b"DICTupdate03", fresh2, sorted=False)
    out["add_fresh_front_ms"] = timed(ix.build_url_ids)
    # 3: a replaced list
    ix.add(idx.hashes[big], rows[1::2].copy())
    out["replace_ms"] = timed(ix.build_url_ids)
    bad, nurls = ix.check_url_ids()
    out["check_bad"] = bad
    out["nurls_after"] = nurls
    os.environ["YRWI_DICT_FULL"] = "1"
    ix.add(b"DICTupdate04", rows[::8].copy())
    out["forced_full_ms"] = timed(ix.build_url_ids)
    out["check_bad_full"] = ix.check_url_ids()[0]
    ix.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
