"""bench.py -- RWI query hot path throughput on MI355X (BASELINE.json metric).

Workload (a "step"): one batch of the C2 query set -- 1000 two-term AND queries,
default RankingProfile, top-100 -- over the synthetic C2 index (10M URLs x 10k
words, 100M postings per GPU), run end to end through libyrwi: join ->
normalise -> cardinal -> top-k, results back in host memory.

N > 1 GPUs (one process per GPU): the index is YaCy's vertical DHT partition
by url hash (Distribution.java:153-158); every rank holds a C2-sized shard of an
N-times larger corpus (weak scaling) and every query runs on all shards, with
RCCL exchanging the normalisation summaries and the per-shard top-k lists.

value = sum over ranks of the postings of all queries (include + exclude list
lengths) / max-over-ranks wall time of the K timed steps.
"""

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from yacy_search_server_amd import RWIIndex, RankingProfile, synth  # noqa: E402
from yacy_search_server_amd._lib import CHit, CQuery, CStats  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def build_queries(idx_hashes, qs, k, now_ms, prof):
    nq = len(qs)
    arr = (CQuery * nq)()
    keep = [prof]
    for i, (inc, exc) in enumerate(qs):
        ib = ctypes.create_string_buffer(b"".join(idx_hashes[t] for t in inc), 12 * max(1, len(inc)))
        eb = ctypes.create_string_buffer(b"".join(idx_hashes[t] for t in exc), 12 * max(1, len(exc)))
        keep += [ib, eb]
        arr[i].incl = ctypes.cast(ib, ctypes.c_void_p)
        arr[i].nincl = len(inc)
        arr[i].excl = ctypes.cast(eb, ctypes.c_void_p)
        arr[i].nexcl = len(exc)
        arr[i].max_distance = 2147483647
        arr[i].k = k
        arr[i].profile = ctypes.pointer(prof.c)
        arr[i].language = b"en"
        arr[i].now_ms = now_ms
    return arr, keep


def cpu_baseline(idx, qs, now_ms, k, budget_s, threads, prof, label, min_s=10.0):
    """The oracle (reference algorithm restated in C++) on a bounded sample of the
    same query stream: one query per thread (ctypes releases the GIL), like the
    GPU's throughput mode.  threads == 1 is the canonical single-thread restatement."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import threading
    import oracle as orc
    oprof = orc.profile_from(prof)
    d = {idx.hashes[t]: idx.list_rows(t) for inc, exc in qs for t in inc + exc if idx.sizes[t]}
    lock = threading.Lock()
    state = {"next": 0, "post": 0, "n": 0}
    t0 = time.perf_counter()

    def worker():
        while True:
            with lock:
                i = state["next"]
                # cycle through the query list until the time budget is spent
                if time.perf_counter() - t0 > budget_s or (i >= len(qs) and time.perf_counter() - t0 > min_s):
                    return
                state["next"] = i + 1
            inc, exc = qs[i % len(qs)]
            orc.search(d, [idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], profile=oprof,
                       now_ms=now_ms, k=k)
            with lock:
                state["post"] += int(sum(idx.sizes[t] for t in inc + exc))
                state["n"] += 1

    ths = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    return {"value": state["post"] / dt, "unit": "postings/s", "cores": threads, "kind": "port",
            "sample": f"{state['n']} queries cycling the {len(qs)} {label} queries ({state['post']} postings, {dt:.1f}s), "
                      f"oracle/yrwi_oracle.cpp, {threads} host thread(s), one query per thread"}


def load_pmc(config):
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--terms", type=int, default=2, help="include terms per query (minimum)")
    ap.add_argument("--max-terms", type=int, default=0, help="include terms per query (maximum; default --terms)")
    ap.add_argument("--exclude", type=int, default=0, help="exclude terms per query")
    ap.add_argument("--profile", default="default", choices=["default", "custom", "date"],
                    help="custom = C5's date=15,domlength=15,authority=13,tf=10; date = the /date modifier")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="(1 GPU) run the rank-0 url-hash shard of a W-GPU corpus: the per-GPU slice of C3/C5")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--latency", type=int, default=100, help="single-query latency samples")
    ap.add_argument("--inflight", type=int, default=2, help="batches in flight (throughput mode)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist

    base = synth.preset(args.config)
    max_terms = max(args.terms, args.max_terms)
    if args.shard_of > 1:
        # the per-GPU slice of a W-GPU corpus (C3/C5 are quoted over 8 GPUs): shard 0 of W
        if world > 1:
            raise SystemExit("--shard-of is a one-GPU option")
        full = base
        cfg = full.shard(0, args.shard_of)
    else:
        # weak scaling: an N-times larger corpus, URL-hash range partitioned over the N ranks
        full = synth.SynthConfig(base.seed, base.n_urls * world, base.n_terms, base.n_hosts * world,
                                 base.n_postings * world)
        cfg = full.shard(rank, world) if world > 1 else full
    t0 = time.time()
    idx = synth.build_index(cfg)
    log(f"rank {rank}: generated {len(idx.rows)} postings in {time.time() - t0:.1f}s")

    if world > 1:
        import torch
        from yacy_search_server_amd import unique_id
        uid = torch.zeros(128, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        ix = RWIIndex(local, shard=(rank, world, bytes(uid.cpu().numpy())))
    else:
        ix = RWIIndex(local)
    t0 = time.time()
    for t in range(cfg.n_terms):
        if idx.sizes[t]:
            ix.add(idx.hashes[t], idx.list_rows(t))
    log(f"rank {rank}: index resident in {time.time() - t0:.1f}s, stats {ix.stats()}")
    t0 = time.time()
    ix.build_url_ids()
    t_dict = time.time() - t0
    log(f"rank {rank}: url dictionary built in {t_dict:.3f}s")

    qs = synth.queries(full, args.nq, args.terms, max_terms, args.exclude)
    now_ms = 20741 * 86400000
    prof = RankingProfile()
    if args.profile == "custom":  # exercises the authority path (coeff > 12)
        prof.coeff_date, prof.coeff_domlength, prof.coeff_authority, prof.coeff_termfrequency = 15, 15, 13, 10
    elif args.profile == "date":
        prof = RankingProfile.date()
    cq, keep = build_queries(idx.hashes, qs, args.k, now_ms, prof)
    kmax = args.k
    # throughput mode: up to `inflight` batches in flight (yrwi_query_batch_submit),
    # each on its own lane, results landing in pinned host buffers
    depth = max(1, args.inflight)
    bufs = [(ix.host_array(CHit, args.nq * kmax), ix.host_array(ctypes.c_int32, args.nq), CStats())
            for _ in range(depth)]
    agg = {"postings_in": 0, "bytes_join": 0, "t_join_ns": 0, "n_join": 0, "bytes_alg": 0, "joined": 0,
           "bytes_probe": 0, "t_probe_ns": 0, "bytes_compact": 0, "t_compact_ns": 0, "t_norm_ns": 0, "t_score_ns": 0, "t_total_ns": 0}
    state = {"depth": depth}

    def collect(st):
        agg["postings_in"] += st.postings_in
        agg["bytes_join"] += st.bytes_join
        agg["t_join_ns"] += st.t_join_ns
        agg["bytes_probe"] += st.bytes_probe
        agg["t_probe_ns"] += st.t_probe_ns
        agg["bytes_compact"] += st.bytes_compact
        agg["t_compact_ns"] += st.t_compact_ns
        agg["n_join"] += st.n_join_launches
        agg["bytes_alg"] += st.bytes_alg
        agg["joined"] += st.joined
        agg["t_norm_ns"] += st.t_norm_ns
        agg["t_score_ns"] += st.t_score_ns
        agg["t_total_ns"] += st.t_total_ns

    def run_steps(n):
        """n steps (batches); every batch is complete (results in host memory) on return."""
        depth = state["depth"]
        pending = []
        for i in range(n):
            b = bufs[i % depth]
            if len(pending) == depth:
                t, bst = pending.pop(0)
                ix.wait(t)
                collect(bst)
            pending.append((ix.submit_raw(cq, args.nq, kmax, b[0], b[1], b[2]), b[2]))
        for t, bst in pending:
            ix.wait(t)
            collect(bst)

    def barrier():
        if dist is not None:
            dist.barrier()

    run_steps(args.warmup)
    for k in agg:
        agg[k] = 0
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize()  # every batch was waited for; this brackets the device too
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        pp = torch.tensor([agg["postings_in"]], dtype=torch.float64, device="cuda")
        dist.all_reduce(pp)
        total_post = float(pp.item())
    else:
        total_post = float(agg["postings_in"])
    value = total_post / dt
    ms_per_step = dt / args.steps * 1e3

    timed = dict(agg)
    # Roofline pass: the same batch, one in flight (no concurrent lane), so the
    # HIP-event duration of each k_join / k_probe launch is that kernel's alone.
    # (In the timed region two lanes overlap and share HBM: "roofline_timed".)
    for k in agg:
        agg[k] = 0
    state["depth"] = 1
    run_steps(max(1, min(args.steps, 5)))
    state["depth"] = depth
    iso = dict(agg)
    iso["batches"] = max(1, min(args.steps, 5))
    pmc = load_pmc(args.config)

    def roofline(a, kernel):
        tkey, bkey = {"k_join": ("t_join_ns", "bytes_join"), "k_probe": ("t_probe_ns", "bytes_probe"),
                      "k_compact": ("t_compact_ns", "bytes_compact")}[kernel]
        t = a[tkey] / max(1, a["n_join"]) * 1e-9
        bpl = a[bkey] / max(1, a["n_join"])
        ach = bpl / t / 1e9 if t > 0 else 0.0
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": pmc.get(f"{kernel}_hbm_bytes_per_launch") if pmc else None,
                "kernel": kernel, "bytes_per_launch_alg": int(bpl), "mean_launch_us": round(t * 1e6, 2)}

    def with_traffic(r):
        if r.get("traffic") and r["mean_launch_us"]:
            r["traffic_GBps"] = round(r["traffic"] / (r["mean_launch_us"] * 1e-6) / 1e9, 1)
            r["traffic_frac"] = round(r["traffic_GBps"] / HBM_PEAK_GBS, 4)
        return r

    # The dominant kernel is k_compact (the row gathers of the joined container):
    # its algorithmic bytes are the rows it must read and write; the PMC traffic
    # beside it shows the sector cost of gathering sparse 40-B rows.
    roof = with_traffic(roofline(iso, "k_compact"))
    roof["measured"] = "HIP events around each launch, separate pass of the timed batch with 1 batch in flight"
    # BASELINE.md §4 counts 12 B per posting key; the join streams 4-byte url ids
    # (DESIGN.md §3), so the HBM bytes it moves are far fewer than its K
    roof_join = with_traffic(roofline(iso, "k_join"))
    roof_probe = with_traffic(roofline(iso, "k_probe"))
    roof_timed = roofline(timed, "k_compact")
    roof_timed["measured"] = "HIP events around each launch inside the timed region (2 lanes overlap)"

    # single-query latency (host call -> top-k in host memory)
    lat = []
    if rank == 0 and world == 1 and args.latency > 0:
        one = (CHit * kmax)()
        n1 = (ctypes.c_int32 * 1)()
        for i in range(min(args.latency, args.nq)):
            t1 = time.perf_counter()
            ix.search_batch_raw(ctypes.byref(cq[i]), 1, kmax, one, n1, CStats())
            lat.append((time.perf_counter() - t1) * 1e3)

    # parity spot check of this very workload: the last batch's hits (pinned host
    # buffers) of the first few queries against the oracle (checker only)
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as orc
        oprof = orc.profile_from(prof)
        hits, nout = bufs[0][0], bufs[0][1]  # the roofline pass above ran last, on bufs[0]
        nchk = min(args.nq, 16)
        bad = 0
        for qi in range(nchk):
            inc, exc = qs[qi]
            d = {idx.hashes[t]: idx.list_rows(t) for t in inc + exc if idx.sizes[t]}
            exp = orc.search(d, [idx.hashes[t] for t in inc], [idx.hashes[t] for t in exc], profile=oprof,
                             now_ms=now_ms, k=args.k)
            got = [(bytes(hits[qi * kmax + j].urlhash), hits[qi * kmax + j].score) for j in range(nout[qi])]
            bad += got != [(h, sc) for h, sc, _ in exp]
        parity = {"queries_checked": nchk, "mismatches": bad, "checker": "oracle/yrwi_oracle.cpp"}
        if bad:
            log(f"PARITY MISMATCH on {bad} of {nchk} queries")

    cpu = cpu1 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        nthr = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))
        cpu = cpu_baseline(idx, qs, now_ms, args.k, args.cpu_budget, nthr, prof, args.config)
        cpu1 = cpu_baseline(idx, qs, now_ms, args.k, args.cpu_budget / 2, 1, prof, args.config)

    if rank == 0:
        terms_s = f"{args.terms}" if max_terms == args.terms else f"{args.terms}-{max_terms}"
        excl_s = f" + {args.exclude} excluded" if args.exclude else ""
        if args.shard_of > 1:
            corpus_s = (f"url-hash shard 0 of {args.shard_of} ({len(idx.rows) / 1e6:.0f}M postings) of the "
                        f"{base.n_postings / 1e6:.0f}M-posting corpus ({base.n_urls / 1e6:.0f}M URLs x "
                        f"{base.n_terms} words)")
        else:
            corpus_s = (f"{base.n_postings / 1e6:.0f}M postings ({base.n_urls / 1e6:.0f}M URLs x "
                        f"{base.n_terms} words) per GPU")
        out = {
            "metric": "postings joined+ranked/sec (node)",
            "value": value, "unit": "postings/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int64", "data": "synthetic",
            "config": {"workload": f"{args.config}: {args.nq} x {terms_s}-term AND queries{excl_s}, "
                                   f"{args.profile} RankingProfile, top-{args.k}; {corpus_s}",
                       "queries_per_step": args.nq, "postings_per_step": total_post / args.steps,
                       "index_postings_total": int(full.n_postings), "parallelism": f"url-hash shards x{world}"},
            "roofline": roof,
            "roofline_join": roof_join,
            "roofline_probe": roof_probe,
            "roofline_timed": roof_timed,
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "cpu_baseline_1thread": cpu1,
            "latency_ms": ({"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                            "n": len(lat)} if lat else None),
            "joined_per_step": timed["joined"] / args.steps,
            "bytes_alg_per_step": timed["bytes_alg"] / args.steps,
            "inflight": args.inflight,
            # per batch, from the library's own HIP events (isolated pass): join+probe kernels,
            # normalisation (reduce..combine), scoring (score..emit); host = call to results
            "phase_ms": {"join": round(iso["t_join_ns"] / 1e6 / max(1, iso["batches"]), 3),
                         "probe": round(iso["t_probe_ns"] / 1e6 / max(1, iso["batches"]), 3),
                         "norm": round(iso["t_norm_ns"] / 1e6 / max(1, iso["batches"]), 3),
                         "score": round(iso["t_score_ns"] / 1e6 / max(1, iso["batches"]), 3),
                         "total": round(iso["t_total_ns"] / 1e6 / max(1, iso["batches"]), 3)},
            "url_dictionary_build_s": round(t_dict, 3),
        }
        print(json.dumps(out))
    ix.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
