"""bench.py -- RWI query hot path throughput on MI355X (BASELINE.json metric).

Headline workload (a "step"): one batch of the C2 query set -- 1000 two-term AND
queries, default RankingProfile, top-100 -- over the synthetic C2 index (10M URLs
x 10k words, 100M postings per GPU), run end to end through libyrwi: join ->
normalise -> cardinal -> top-k, results back in host memory.

N GPUs: `python bench.py --gpus N` starts N rank processes itself (one per GPU,
before anything touches a GPU); under torchrun the ranks come from the
environment.  The index is YaCy's vertical DHT partition by url hash
(Distribution.java:153-158):
  --scaling weak (default)  every rank holds a C2-sized shard of an N-times larger
                            corpus (per-GPU work fixed: the driver's 1/2/4/8 series);
  --scaling strong          the configured corpus (fixed) is split over the N ranks.
Every query runs on every shard; RCCL exchanges the term sizes, the
normalisation summaries and the per-shard top-k lists.

value = sum over ranks of the postings of all queries (include + exclude list
lengths) / max-over-ranks wall time of the K timed steps.

After the headline the default run measures the other BASELINE configs as
extra legs on the same GPUs: C3 (1B postings, 3-term AND + 1
exclude, split over the N ranks: strong scaling), C4 (4096 concurrent 2-4 term
queries over the C3 index) and C5 (the custom and /date RankingProfiles over the
per-GPU 625M-posting slice of the 5B corpus).  `--legs none` skips them.
"""

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
NOW_MS = 20741 * 86400000


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--terms", type=int, default=2, help="include terms per query (minimum)")
    ap.add_argument("--max-terms", type=int, default=0, help="include terms per query (maximum; default --terms)")
    ap.add_argument("--exclude", type=int, default=0, help="exclude terms per query")
    ap.add_argument("--qseed", type=lambda x: int(x, 0), default=None,
                    help="query stream seed (default: the config's; C4 uses seed ^ 0xC4)")
    ap.add_argument("--profile", default="default", choices=["default", "custom", "date"],
                    help="custom = C5's date=15,domlength=15,authority=13,tf=10; date = the /date modifier")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--shard-of", type=int, default=1,
                    help="(1 GPU) run the rank-0 url-hash shard of a W-GPU corpus: the per-GPU slice of C3/C5")
    ap.add_argument("--legs", default="auto",
                    help="extra BASELINE configs after the headline ('C3,C4,C5'), or 'none'; "
                         "auto: C3,C4,C5 on one GPU, none for N > 1 (the scaling runs time the headline only)")
    ap.add_argument("--leg-steps", type=int, default=20)
    ap.add_argument("--leg-check", type=int, default=4,
                    help="queries of each distinct batch of a leg's timed region checked against the oracle")
    ap.add_argument("--check", type=int, default=16,
                    help="queries of each distinct batch of the headline's timed region checked against the oracle")
    ap.add_argument("--batches", type=int, default=8,
                    help="distinct query batches cycled over the timed steps (one per in-flight slot; "
                         "capped at --inflight and made to divide it)")
    ap.add_argument("--leg-latency", type=int, default=50, help="single-query latency samples per leg")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--latency", type=int, default=100, help="single-query latency samples")
    ap.add_argument("--inflight", type=int, default=8, help="batches in flight (throughput mode; the library runs 8 lanes)")
    ap.add_argument("--dry-run", action="store_true", help="ranks + rendezvous only (gloo, no GPU): launcher test")
    return ap.parse_args(argv)


# --------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int) -> int:
    """One process per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in the
    environment), started as children before anything here touches a GPU."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc), 0)


# ------------------------------------------------------------------ provenance
_IDENT = None


def source_identity():
    """Which build this is: `src` = sha1 (12 hex) of libyrwi's sources (csrc/ and
    include/yrwi.h) -- the same on the GPU box, which has no .git; `head` = the git
    commit (here) or the REVISION file a post-commit hook leaves in the tree (box).
    tools/pmc_summary.py stamps profiles with the same pair, so a bench line can
    say whether its counter profile measured this very build."""
    global _IDENT
    if _IDENT is None:
        import hashlib
        h = hashlib.sha1()
        csrc = os.path.join(ROOT, "yacy_search_server_amd", "csrc")
        files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                       if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile")
        for p in files + [os.path.join(ROOT, "include", "yrwi.h")]:
            h.update(os.path.basename(p).encode())
            with open(p, "rb") as f:
                h.update(f.read())
        head = None
        try:
            head = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], text=True,
                                           stderr=subprocess.DEVNULL).strip() or None
        except (OSError, subprocess.CalledProcessError):
            pass
        if head is None and os.path.exists(os.path.join(ROOT, "REVISION")):
            with open(os.path.join(ROOT, "REVISION")) as f:
                head = f.read().strip() or None
        _IDENT = {"head": head, "src": h.hexdigest()[:12]}
    return _IDENT


# ------------------------------------------------------------------- baselines
def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpus():
    """CPUs' worth of time the cgroup grants this job (cpu.max quota / period), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(q) // int(per))
    except (OSError, ValueError):
        return None


def cgroup_cpu_stat():
    """The job's cgroup CPU accounting (usage / throttling counters), or None."""
    try:
        out = {}
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                out[k] = int(v)
        return out
    except (OSError, ValueError):
        return None


def host_cores():
    """(threads used, affinity cores, why): every core of this process's affinity,
    capped by what the job may actually use -- the cgroup CPU quota (cpu.max) and
    the host-thread share the machine gives this job (OMP_NUM_THREADS / MAX_JOBS,
    the per-GPU share on the GPU boxes).  More threads than the quota only
    time-slice the same CPUs."""
    aff = len(os.sched_getaffinity(0))
    caps = [(int(os.environ[v]), f"{v}={os.environ[v]}") for v in ("OMP_NUM_THREADS", "MAX_JOBS")
            if os.environ.get(v, "").isdigit()]
    q = cgroup_cpus()
    if q is not None:
        caps.append((q, f"cgroup cpu.max quota of {q} CPUs"))
    caps = [c for c in caps if c[0] < aff]
    if caps:
        n, why = min(caps)
        return n, aff, f"{why} of {aff} affinity cores"
    return aff, aff, "all affinity cores"


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
            "cpu_model": cpu_model(),
            "sample": f"{state['n']} queries cycling the {len(qs)} {label} queries ({state['post']} postings, {dt:.1f}s), "
                      f"oracle/yrwi_oracle.cpp, {threads} host thread(s), one query per thread"}


def draws(cfg, nq, min_incl, max_incl, n_excl, qseed, n):
    """n distinct query batches of one stream shape: batch 0 with `qseed` (None: the
    config's default), batch b > 0 with a seed of its own (the same df-proportional
    term sampling)."""
    from yacy_search_server_amd import synth
    base = qseed if qseed is not None else cfg.seed ^ 0x51
    return [synth.queries(cfg, nq, min_incl, max_incl, n_excl,
                          qseed=base if b == 0 else (base + 0x9E3779B97F4A7C15 * b) & 0xFFFFFFFFFFFFFFFF)
            for b in range(max(1, n))]


def load_pmc(config):
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if os.path.exists(path):
        with open(path) as f:
            d = json.load(f)
        d["_file"] = os.path.relpath(path, ROOT)
        return d
    return None


# ------------------------------------------------------------------ the runner
class Runner:
    """One index resident on this rank's GPU and query batches run over it."""

    def __init__(self, args, rank, world, local, dist):
        self.args, self.rank, self.world, self.local, self.dist = args, rank, world, local, dist
        self.ix = None

    def transports(self):
        """Every rank's yrwi_shard_info (rank order), gathered over the job's process group."""
        if self.dist is None:
            return None
        infos = [None] * self.world
        self.dist.all_gather_object(infos, getattr(self, "transport", None))
        return infos

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def open_index(self, cfg):
        from yacy_search_server_amd import RWIIndex, synth, unique_id
        t0 = time.time()
        idx = synth.build_index(cfg)
        log(f"rank {self.rank}: generated {len(idx.rows)} postings in {time.time() - t0:.1f}s")
        if self.world > 1:
            import torch
            uid = torch.zeros(128, dtype=torch.uint8, device="cuda")
            if self.rank == 0:
                uid.copy_(torch.frombuffer(bytearray(unique_id()), dtype=torch.uint8))
            self.dist.broadcast(uid, 0)
            ix = RWIIndex(self.local, shard=(self.rank, self.world, bytes(uid.cpu().numpy())))
            self.transport = ix.shard_info()
            log(f"rank {self.rank}: shard transport {self.transport}")
        else:
            ix = RWIIndex(self.local)
        t0 = time.time()
        for t in range(cfg.n_terms):
            if idx.sizes[t]:
                ix.add(idx.hashes[t], idx.list_rows(t))
        log(f"rank {self.rank}: index resident in {time.time() - t0:.1f}s, stats {ix.stats()}")
        t0 = time.time()
        ix.build_url_ids()
        t_dict = time.time() - t0
        log(f"rank {self.rank}: url dictionary and ranking records built in {t_dict:.3f}s")
        self.ix = ix
        return idx, t_dict

    def close(self):
        if self.ix is not None:
            self.ix.close()
            self.ix = None

    def measure(self, batches, hashes, prof, k, steps, warmup, inflight, isolated=True, identical=True):
        """`batches`: D distinct query batches of the same shape (draws of one query
        stream).  Untimed: every batch once with statistics (its postings and bytes),
        then `warmup` steps.  Timed: `steps` batches, step i = batch i % D in the
        in-flight slot i % inflight (D divides inflight), max over ranks; the timed
        region's own output buffers are copied out right after it (the parity
        sample checks them).  Then, untimed against the headline: the same region
        with one batch every step (`identical`), and an isolated pass (one batch
        in flight) whose library statistics give the per-kernel times."""
        import ctypes
        import torch
        from yacy_search_server_amd import _lib
        from yacy_search_server_amd._lib import CHit, CQuery, CStats
        ix = self.ix
        nq = len(batches[0])
        depth = max(1, inflight)
        D = max(1, min(len(batches), depth))
        while depth % D:
            D -= 1
        batches = batches[:D]
        keep = [prof]
        arrs = []
        for qs in batches:
            arr = (CQuery * nq)()
            for i, (inc, exc) in enumerate(qs):
                ib = ctypes.create_string_buffer(b"".join(hashes[t] for t in inc), 12 * max(1, len(inc)))
                eb = ctypes.create_string_buffer(b"".join(hashes[t] for t in exc), 12 * max(1, len(exc)))
                keep += [ib, eb]
                arr[i].incl = ctypes.cast(ib, ctypes.c_void_p)
                arr[i].nincl = len(inc)
                arr[i].excl = ctypes.cast(eb, ctypes.c_void_p)
                arr[i].nexcl = len(exc)
                arr[i].max_distance = 2147483647
                arr[i].k = k
                arr[i].profile = ctypes.pointer(prof.c)
                arr[i].language = b"en"
                arr[i].now_ms = NOW_MS
            arrs.append(arr)
        bufs = [(ix.host_array(CHit, nq * k), ix.host_array(ctypes.c_int32, nq), CStats()) for _ in range(depth)]
        fields = [f for f, _ in CStats._fields_ if f != "reserved"]
        agg = {f: 0 for f in fields}
        per_batch = [None] * D
        state = {"depth": depth}

        def collect(st, bi):
            for f in fields:
                agg[f] += getattr(st, f)
            per_batch[bi] = {f: getattr(st, f) for f in fields}

        trace = os.environ.get("YRWI_BENCH_TRACE")  # per-batch completion times to stderr

        def run_steps(n, stats=True, batch_of=lambda i: i % D):
            d = state["depth"]
            pending = []
            tl = [time.perf_counter()]
            for i in range(n):
                b = bufs[i % d]
                if len(pending) == d:
                    t, bst, bi = pending.pop(0)
                    ix.wait(t)
                    if bst is not None:
                        collect(bst, bi)
                    tl.append(time.perf_counter())
                st = b[2] if stats else None
                bi = batch_of(i)
                pending.append((ix.submit_raw(arrs[bi], nq, k, b[0], b[1], st), st, bi))
            for t, bst, bi in pending:
                ix.wait(t)
                if bst is not None:
                    collect(bst, bi)
                tl.append(time.perf_counter())
            if trace:
                log("batch done at ms: " + " ".join(f"{(x - tl[0]) * 1e3:.2f}" for x in tl[1:]))

        def timed_region(n, stats, batch_of):
            for f in agg:
                agg[f] = 0
            self.barrier()
            torch.cuda.synchronize()
            r0 = _lib.lib().yrwi_realloc_events()
            cs0 = cgroup_cpu_stat()
            t0 = time.perf_counter()
            run_steps(n, stats=stats, batch_of=batch_of)
            torch.cuda.synchronize()  # every batch was waited for; this brackets the device too
            self.barrier()
            dt = time.perf_counter() - t0
            realloc = int(_lib.lib().yrwi_realloc_events() - r0)  # process-wide, no HIP events needed
            cs1 = cgroup_cpu_stat()
            throttle = {x: cs1[x] - cs0[x] for x in cs0 if x in cs1} if cs0 and cs1 else None
            if not stats:  # the batches' counts from their statistics run
                for f in agg:
                    agg[f] = sum(per_batch[batch_of(i)][f] for i in range(n)) if f != "n_realloc" else 0
            agg["n_realloc"] = realloc
            return dt, dict(agg), throttle

        def over_ranks(dt, post):
            if self.dist is None:
                return dt, post
            tt = torch.tensor([dt, post], dtype=torch.float64, device="cuda")
            tmax = tt[:1].clone()
            self.dist.all_reduce(tmax, op=self.dist.ReduceOp.MAX)
            self.dist.all_reduce(tt)
            return float(tmax.item()), float(tt[1].item())

        # every distinct batch once with statistics (in flight like the timed steps), then
        # every lane's scratch and staging sized to the largest of them (yrwi_settle_scratch:
        # no lane grows on its first large batch inside the timed region), then the warm-up
        run_steps(D)
        rc = _lib.lib().yrwi_settle_scratch(ix._h)
        if rc:
            raise RuntimeError(f"yrwi_settle_scratch: {rc}")
        run_steps(warmup)
        # timed region without per-batch statistics (no HIP events, as a production
        # caller runs); YRWI_BENCH_STATS=1 collects them in the timed region
        timed_stats = os.environ.get("YRWI_BENCH_STATS", "0") == "1"
        gap = float(os.environ.get("YRWI_BENCH_GAP_MS", "0"))  # diagnosis: idle time before the timed region
        if gap > 0:
            time.sleep(gap / 1e3)
        dt, timed, throttle = timed_region(steps, timed_stats, lambda i: i % D)
        if gap > 0:  # (diagnosis: the same idle time after it, so a kernel trace shows where it ends)
            time.sleep(gap / 1e3)
        dt, total_post = over_ranks(dt, float(timed["postings_in"]))
        # the timed region's own results: slot s last ran step i_s (batch i_s % D)
        out = {}
        for s in range(min(depth, steps)):
            i_last = max(i for i in range(steps) if i % depth == s)
            bi = i_last % D
            if bi not in out:
                out[bi] = (bytes(memoryview(bufs[s][0]).cast("B")), list(bufs[s][1]))
        timed["stats_in_timed_region"] = timed_stats
        timed["cgroup_cpu_stat"] = throttle
        ident = None
        if identical and D > 1:
            dt1, t1, _ = timed_region(steps, timed_stats, lambda i: 0)
            dt1, post1 = over_ranks(dt1, float(t1["postings_in"]))
            ident = {"ms_per_step": dt1 / steps * 1e3, "value": post1 / dt1, "realloc_events": t1["n_realloc"],
                     "what": f"the same timed region with batch 0 at every step ({steps} steps, "
                             f"{depth} in flight): eight lanes run identical batches at once"}
        iso = None
        if isolated:
            # batch 0 with one in flight: the library's HIP-event times are then each
            # kernel's alone (in the timed region several lanes share the GPU); five
            # single batches, the one with the median kernel time stands for all (a
            # host stall inside a group of launches would inflate a mean)
            state["depth"] = 1
            runs = []
            for _ in range(max(1, min(steps, 5))):
                for f in agg:
                    agg[f] = 0
                run_steps(1, batch_of=lambda i: 0)
                runs.append(dict(agg))
            runs.sort(key=lambda r: r["t_kernels_ns"])
            iso = runs[len(runs) // 2]
            iso["batches"] = 1
            iso["isolated_runs_t_kernels_us"] = [round(r["t_kernels_ns"] / 1e3, 1) for r in runs]
        return {"dt": dt, "steps": steps, "total_post": total_post, "timed": timed, "iso": iso, "bufs": bufs,
                "arrs": arrs, "keep": keep, "timed_out": out, "batches": batches, "D": D, "identical": ident,
                "per_batch_postings": [pb["postings_in"] for pb in per_batch]}


def check_and_latency(R, M, hashes, idx, prof, k, nchk, nlat, label, threads=1):
    """Outside the timed region: (a) `nchk` queries (evenly spaced) of EVERY distinct
    batch, read from the timed region's own output buffers (copied right after
    it), against the oracle (checker only, oracle/yrwi_oracle.cpp; `threads`
    queries at a time, ctypes releases the GIL); (b) host-call ->
    top-k-in-host-memory latency of `nlat` single queries of batch 0, no
    statistics (the production call)."""
    import ctypes
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from yacy_search_server_amd._lib import CHit
    parity = None
    if nchk > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as orc
        oprof = orc.profile_from(prof)
        hsz = ctypes.sizeof(CHit)
        jobs = []
        for bi, qs in enumerate(M["batches"]):
            nq = len(qs)
            if bi not in M["timed_out"]:
                continue
            raw, nout = M["timed_out"][bi]
            hits = (CHit * (nq * k)).from_buffer_copy(raw)
            for qi in sorted({i * nq // min(nchk, nq) for i in range(min(nchk, nq))}):
                got = [(bytes(hits[qi * k + j].urlhash), hits[qi * k + j].score) for j in range(nout[qi])]
                jobs.append((bi, qi, qs[qi], got))

        def one(job):
            bi, qi, (inc, exc), got = job
            d = {hashes[t]: idx.list_rows(t) for t in inc + exc if idx.sizes[t]}
            exp = orc.search(d, [hashes[t] for t in inc], [hashes[t] for t in exc], profile=oprof,
                             now_ms=NOW_MS, k=k)
            return None if got == [(h, sc) for h, sc, _ in exp] else (bi, qi)

        with ThreadPoolExecutor(max(1, threads)) as ex:
            bad = [r for r in ex.map(one, jobs) if r is not None]
        parity = {"queries_checked": len(jobs), "mismatches": len(bad), "checker": "oracle/yrwi_oracle.cpp",
                  "distinct_batches_checked": len(M["timed_out"]),
                  "queries": f"{nchk} evenly spaced queries of each of the {len(M['timed_out'])} distinct batches, "
                             f"read from the timed region's own output buffers (no statistics, the production call)"}
        if bad:
            log(f"{label}: PARITY MISMATCH on (batch, query) {bad[:10]}")
    lat = None
    if nlat > 0:
        one_h = (CHit * k)()
        n1 = (ctypes.c_int32 * 1)()
        arr = M["arrs"][0]
        ts = []
        for i in range(min(nlat, len(M["batches"][0]))):
            t1 = time.perf_counter()
            R.ix.search_batch_raw(ctypes.byref(arr[i]), 1, k, one_h, n1, None)
            ts.append((time.perf_counter() - t1) * 1e3)
        lat = {"p50": float(np.percentile(ts, 50)), "p99": float(np.percentile(ts, 99)), "n": len(ts),
               "what": "one query per call (yrwi_query_batch, nq = 1, no statistics): host call -> top-k in host memory"}
    return parity, lat


def _frac(gbps):
    """Fraction of the HBM peak, or None when the byte model's rate passes the peak
    (then the model credits reads the kernel never makes: no fraction is claimed)."""
    return round(gbps / HBM_PEAK_GBS, 4) if 0 < gbps <= HBM_PEAK_GBS else None


def kernel_lines(iso, pmc):
    """Every path kernel that moves the batch's postings, each on its bytes over its
    mean launch time (library HIP events around each launch, isolated pass):
      k_join    SURVEY.md §8(d): sum of min(K, 4-B ids of both sides) over the merge-executed steps;
      k_probe   §8(d): sum of min(K, bytes the probe loads) over the probe-executed include steps
                (url-id bitmap: 4-B id + one 16-B bitmap word per smaller-side id); K as the reference
                dispatches the step (J3);
      k_compact §8(d): 23 B per include term and joined posting (23 t m_out);
      k_reduce  the 32-B ranking record of every joined posting the compaction did not summarise
                (+ 1-B exclusion mark); its time includes k_piece_merge (the compaction's pieces,
                no container read: 0 bytes when every query has them);
      k_score   the same records (an upper bound: chunks the threshold prunes read 16 of the 32 B);
      k_chain   §8(d): the chained folds' later steps' K and the exclusions' 12 n_e, each charged
                min(K, the bytes k_chain loads for it) (k_chain_part and k_scan_tiles included).
    traffic = rocprofv3 PMC HBM bytes per launch (profiles/pmc_<config>.json) and
    hbm_frac = traffic / the profile's own mean launch time / peak (the same dispatches)."""
    n = max(1, iso["n_join_launches"])
    nr = max(1, iso.get("n_rank_passes", 0))
    pk = (pmc or {}).get("kernels", {})
    out = {}
    for name, t_ns, alg, nl, extra in (
            ("k_join", iso["t_join_ns"], iso["bytes_join_capped"], n,
             {"alg_bytes_model_K": int(iso["bytes_join"] / n)}),
            ("k_probe", iso["t_probe_ns"], iso["bytes_probe_capped"], n,
             {"alg_bytes_model_K": int(iso["bytes_probe"] / n), "loaded_bytes": int(iso["bytes_probe_loaded"] / n)}),
            ("k_compact", iso["t_compact_ns"], iso["bytes_features"], n, {}),
            ("k_reduce", iso.get("t_reduce_ns", 0), iso.get("bytes_reduce", 0), nr, {}),
            ("k_score", iso.get("t_scorek_ns", 0), iso.get("bytes_score", 0), nr, {}),
            ("k_chain", iso.get("t_chain_ns", 0), iso.get("bytes_chain", 0), max(1, iso.get("n_chain_launches", 0)),
             {})):
        t = t_ns / nl * 1e-9
        if t <= 0:
            continue
        a = alg / nl
        # (the compaction: k_compact and / or k_compact_sum per step, pooled by tools/pmc_summary.py)
        kd = pk.get("compaction", pk.get(name, {})) if name == "k_compact" else pk.get(name, {})
        traffic = kd.get("hbm_bytes_per_launch")
        # bytes credited: the SURVEY 8(d) model, capped at the bytes the counters saw
        # leave L2 (a model above them credits requests L2 / LDS served)
        cred = min(a, traffic) if traffic else a
        gbps = cred / t / 1e9
        e = {"mean_launch_us": round(t * 1e6, 2), "alg_bytes": int(a), "credited_bytes": int(cred),
             "capped_at_traffic": bool(traffic and a > traffic), "achieved": round(gbps, 1), "frac": _frac(gbps)}
        e.update(extra)
        if name == "k_reduce" and not alg:
            e["note"] = "k_piece_merge only: every query's container was summarised by k_compact_sum"
        if name == "k_probe" and iso.get("n_probe_dispatches"):
            # every k_probe dispatch, the exclusion steps' too (profiles key those as k_probe_excl)
            e["mean_dispatch_us_all_steps"] = round(iso["t_probe_all_ns"] / iso["n_probe_dispatches"] / 1e3, 2)
        if traffic:
            e["traffic"] = traffic
            e["traffic_GBps"] = round(traffic / t / 1e9, 1)
            tp = kd.get("avg_ns", 0) * 1e-9
            if tp > 0:
                e["rocprof_mean_launch_us"] = round(tp * 1e6, 2)
                e["frac_rocprof"] = _frac(cred / tp / 1e9)
                e["hbm_frac"] = round(traffic / tp / 1e9 / HBM_PEAK_GBS, 4)
            if kd.get("read_requests_dram_per_launch") is not None:
                e["dram_read_bytes"] = round(128 * kd["read_requests_dram_per_launch"])
        out[name] = e
    return out


def roofline_block(iso, timed, steps, ms_per_step, pmc):
    """`roofline` of the bench line: the dominant kernel (longest mean launch among
    every path kernel of kernel_lines) with its bytes, plus the path: B = sum K +
    12 sum n_excl + 23 t m_out per batch with every join and exclusion step
    charged min(K, the bytes its kernel loads), over (a) the batch's kernel time in
    the isolated pass and (b) the timed region's time per batch (batches in flight
    overlap)."""
    kern = kernel_lines(iso, pmc)
    nb = max(1, iso["batches"])
    if not kern:
        return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None}, kern
    dom = max(kern, key=lambda k: kern[k]["mean_launch_us"])
    d = kern[dom]
    r = {"bound": "hbm", "kernel": dom, "achieved": d["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": d["frac"], "traffic": d.get("traffic"), "hbm_frac": d.get("hbm_frac"),
         "alg_bytes_per_launch": d["alg_bytes"], "credited_bytes_per_launch": d["credited_bytes"],
         "mean_launch_us": d["mean_launch_us"],
         "measured": "HIP events around each launch on the lane's stream (library statistics), isolated pass "
                     "(one batch in flight, median of five batches)"}
    if d.get("rocprof_mean_launch_us"):
        r["rocprof_mean_launch_us"] = d["rocprof_mean_launch_us"]
        r["frac_rocprof"] = d.get("frac_rocprof")
    if d.get("mean_dispatch_us_all_steps"):
        r["mean_dispatch_us_all_steps"] = d["mean_dispatch_us_all_steps"]
    if pmc:
        r["traffic_source"] = (f"{pmc['_file']} (rocprofv3 --pmc: TCC_EA0_RDREQ_32B/64B/128B, TCC_EA0_WRREQ/_64B "
                               f"by request size, each pass its own run; hbm_frac over the same profile's "
                               f"kernel-trace mean; tag {pmc.get('tag')}, commit {pmc.get('head')})")
        r["profile"] = {"file": pmc["_file"], "head": pmc.get("head"), "src": pmc.get("src"),
                        "src_match": pmc.get("src") == source_identity()["src"]}
    b_iso = iso["bytes_alg_capped"] / nb
    t_iso = iso["t_kernels_ns"] / nb * 1e-9
    path = {"bytes_per_batch": int(b_iso),
            "bytes_per_batch_model": int(iso["bytes_alg"] / nb),
            "rule": "SURVEY 8(d) B with every join / exclusion step charged min(K, the bytes its kernel loads)"}
    if t_iso > 0:
        g = b_iso / t_iso / 1e9
        path["isolated"] = {"achieved": round(g, 1), "frac": _frac(g), "kernel_us_per_batch": round(t_iso * 1e6, 1)}
        if iso.get("isolated_runs_t_kernels_us"):
            path["isolated"]["batches_kernel_us"] = iso["isolated_runs_t_kernels_us"]
    if timed.get("bytes_alg") and ms_per_step > 0:
        bt = timed["bytes_alg_capped"] / steps
        g = bt / (ms_per_step * 1e-3) / 1e9
        path["throughput_mode"] = {"achieved": round(g, 1), "frac": _frac(g), "per": "GPU",
                                   "time": "ms_per_step (timed region, batches in flight)"}
    if pmc and pmc.get("path_hbm_bytes_per_batch"):
        path["traffic_per_batch"] = pmc["path_hbm_bytes_per_batch"]
        if t_iso > 0:
            path["isolated"]["hbm_frac"] = round(pmc["path_hbm_bytes_per_batch"] / t_iso / 1e9 / HBM_PEAK_GBS, 4)
        if ms_per_step > 0:
            path["throughput_mode"]["hbm_frac"] = round(
                pmc["path_hbm_bytes_per_batch"] / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    r["path"] = path
    return r, kern


def run(args, rank, world, local):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from yacy_search_server_amd import RankingProfile, synth

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist
    R = Runner(args, rank, world, local, dist)

    base = synth.preset(args.config)
    max_terms = max(args.terms, args.max_terms)
    if args.shard_of > 1:
        # the per-GPU slice of a W-GPU corpus (C3/C5 are quoted over 8 GPUs): shard 0 of W
        if world > 1:
            raise SystemExit("--shard-of is a one-GPU option")
        full = base
        cfg = full.shard(0, args.shard_of)
    elif args.scaling == "strong":
        full = base
        cfg = full.shard(rank, world) if world > 1 else full
    else:
        # weak scaling: an N-times larger corpus, URL-hash range partitioned over the N ranks
        full = synth.SynthConfig(base.seed, base.n_urls * world, base.n_terms, base.n_hosts * world,
                                 base.n_postings * world)
        cfg = full.shard(rank, world) if world > 1 else full
    idx, t_dict = R.open_index(cfg)

    bats = draws(full, args.nq, args.terms, max_terms, args.exclude, args.qseed, args.batches)
    qs = [q for b in bats for q in b]  # the CPU baseline cycles every distinct batch's queries
    prof = RankingProfile()
    if args.profile == "custom":  # exercises the authority path (coeff > 12)
        prof.coeff_date, prof.coeff_domlength, prof.coeff_authority, prof.coeff_termfrequency = 15, 15, 13, 10
    elif args.profile == "date":
        prof = RankingProfile.date()
    shard_transport = transport_summary(R.transports()) if world > 1 else None
    M = R.measure(bats, idx.hashes, prof, args.k, args.steps, args.warmup, args.inflight)
    value = M["total_post"] / M["dt"]
    ms_per_step = M["dt"] / args.steps * 1e3
    iso, timed = M["iso"], M["timed"]
    pmc = load_pmc(args.config) if world == 1 and args.shard_of == 1 else None
    roof, kern = roofline_block(iso, timed, args.steps, ms_per_step, pmc)

    # parity of this very workload and single-query latency (outside the timed region)
    parity = lat = None
    if rank == 0 and world == 1:
        parity, lat = check_and_latency(R, M, idx.hashes, idx, prof, args.k, 0 if args.no_cpu else args.check,
                                        args.latency, args.config, threads=host_cores()[0])

    cpu = cpu1 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        nthr, aff, why = host_cores()
        cpu = cpu_baseline(idx, qs, NOW_MS, args.k, args.cpu_budget, nthr, prof, args.config)
        cpu["cores_why"] = why
        cpu["affinity_cores"] = aff
        cpu["cgroup_cpus"] = cgroup_cpus()
        cpu1 = cpu_baseline(idx, qs, NOW_MS, args.k, args.cpu_budget / 2, 1, prof, args.config)
    R.close()
    shard_postings = len(idx.rows)
    del idx

    legs = {}
    if args.legs == "auto":
        args.legs = "C3,C4,C5" if world == 1 else "none"
    if args.legs and args.legs != "none" and args.shard_of == 1:
        for leg in [x.strip() for x in args.legs.split(",") if x.strip()]:
            try:
                legs.update(run_leg(R, leg, args, rank, world))
            except Exception as e:  # a leg never sinks the headline line
                log(f"leg {leg} failed: {e!r}")
                legs[leg] = {"error": repr(e)}
                R.close()

    if rank == 0:
        terms_s = f"{args.terms}" if max_terms == args.terms else f"{args.terms}-{max_terms}"
        excl_s = f" + {args.exclude} excluded" if args.exclude else ""
        if args.shard_of > 1:
            corpus_s = (f"url-hash shard 0 of {args.shard_of} ({shard_postings / 1e6:.0f}M postings) of the "
                        f"{base.n_postings / 1e6:.0f}M-posting corpus ({base.n_urls / 1e6:.0f}M URLs x "
                        f"{base.n_terms} words)")
        elif args.scaling == "strong":
            corpus_s = (f"{base.n_postings / 1e6:.0f}M postings ({base.n_urls / 1e6:.0f}M URLs x {base.n_terms} words) "
                        f"split over {world} GPU(s)")
        else:
            corpus_s = (f"{base.n_postings / 1e6:.0f}M postings ({base.n_urls / 1e6:.0f}M URLs x "
                        f"{base.n_terms} words) per GPU")
        nbi = max(1, iso["batches"])
        out = {
            "metric": "postings joined+ranked/sec (node)",
            "value": value, "unit": "postings/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "int64", "data": "synthetic",
            "config": {"workload": f"{args.config}: {args.nq} x {terms_s}-term AND queries{excl_s}, "
                                   f"{args.profile} RankingProfile, top-{args.k}; {corpus_s}",
                       "queries_per_step": args.nq, "postings_per_step": M["total_post"] / args.steps,
                       "index_postings_total": int(full.n_postings), "parallelism": f"url-hash shards x{world}"},
            "roofline": roof,
            "roofline_kernels": kern,
            "cpu_baseline": cpu,
            "cpu_baseline_1thread": cpu1,
            "parity_sample": parity,
            "latency_ms": lat,
            "joined_per_step": timed["joined"] / args.steps,
            "bytes_alg_per_step": timed["bytes_alg"] / args.steps,
            # device-wide allocation events (scratch / pinned staging growth) inside the timed steps
            "realloc_events_timed": timed["n_realloc"],
            # the job's CPU-quota accounting over the timed region (cgroup cpu.stat deltas)
            "cgroup_cpu_stat_timed": timed.get("cgroup_cpu_stat"),
            "timed_region": ("batches submitted with per-batch statistics (YRWI_BENCH_STATS=1)"
                             if timed["stats_in_timed_region"] else
                             "batches submitted without statistics (no HIP events: the production call); "
                             "postings and bytes of each distinct batch from its statistics run before the warm-up"),
            "distinct_batches": M["D"],
            "batch_schedule": f"step i runs distinct batch i % {M['D']} in in-flight slot i % {args.inflight}",
            "postings_per_batch": M["per_batch_postings"],
            "identical_batch": M["identical"],
            "inflight": args.inflight,
            # per batch, from the library's own HIP events (isolated pass): join+probe kernels,
            # normalisation (reduce..combine), scoring (score..emit), all kernels; host = call to results
            "phase_ms": phase_ms(iso),
            "url_dictionary_build_s": round(t_dict, 3),
            "legs": legs or None,
            # world > 1: how the shards' collectives travelled (yrwi_shard_info of every rank)
            "shard_transport": shard_transport,
        }
        ident = source_identity()
        out["build"] = ident
        detail = write_detail(out, ident)
        print(json.dumps(compact_line(out, detail)), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def write_detail(out, ident):
    """The full record (every per-kernel block, the path model, the identical-batch
    run, per-batch data) goes to profiles/bench_detail_src<source hash>.json and, when a
    gpurun_out/ directory can be made, a copy there (what a GPU call brings back)."""
    # named by the hash of libyrwi's sources: the committed detail of a build's own
    # full run carries the same name as any later run of that build (the driver's)
    name = f"bench_detail_src{ident['src']}.json"
    rel = os.path.join("profiles", name)
    for d in (os.path.join(ROOT, "profiles"), os.path.join(ROOT, "gpurun_out")):
        try:
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, name), "w") as f:
                json.dump(out, f, indent=1)
        except OSError as e:
            log(f"detail not written to {d}: {e!r}")
    return rel


def _short_roof(r):
    keep = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "hbm_frac", "alg_bytes_per_launch",
            "credited_bytes_per_launch", "mean_launch_us", "rocprof_mean_launch_us", "frac_rocprof")
    o = {k: r.get(k) for k in keep if k in r}
    if r.get("profile"):
        o["profile"] = r["profile"]
    p = r.get("path") or {}
    if p:
        o["path"] = {"bytes_per_batch": p.get("bytes_per_batch"), "traffic_per_batch": p.get("traffic_per_batch"),
                     "isolated_frac": (p.get("isolated") or {}).get("frac"),
                     "throughput_frac": (p.get("throughput_mode") or {}).get("frac"),
                     "throughput_hbm_frac": (p.get("throughput_mode") or {}).get("hbm_frac")}
    return o


def _short_leg(leg):
    if "error" in leg:
        return {"error": leg["error"][:200]}
    r = leg.get("roofline") or {}
    par = leg.get("parity_sample") or {}
    lat = leg.get("latency_ms") or {}
    return {"ms_per_step": round(leg["ms_per_step"], 4), "value": leg["value"], "kernel": r.get("kernel"),
            "frac": r.get("frac"), "frac_rocprof": r.get("frac_rocprof"), "hbm_frac": r.get("hbm_frac"),
            "checked": par.get("queries_checked"), "mismatches": par.get("mismatches"),
            "p50_ms": round(lat["p50"], 3) if lat.get("p50") is not None else None,
            "realloc_events_timed": leg.get("realloc_events_timed")}


def compact_line(out, detail):
    """The one stdout line the driver parses (kept to a few KB: round 4's 20 KB line
    overflowed the driver's tail).  The full record is in `detail`."""
    cpu = out.get("cpu_baseline")
    cpu1 = out.get("cpu_baseline_1thread")
    par = out.get("parity_sample")
    lat = out.get("latency_ms")
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")}
    line["roofline"] = _short_roof(out["roofline"])
    line["cpu_baseline"] = None if cpu is None else {
        "value": cpu["value"], "unit": cpu["unit"], "cores": cpu["cores"], "kind": cpu["kind"],
        "sample": cpu["sample"], "cpu_model": cpu.get("cpu_model")}
    line["cpu_baseline_1thread"] = None if cpu1 is None else {"value": cpu1["value"], "cores": cpu1["cores"]}
    line["parity_sample"] = None if par is None else {
        "queries_checked": par["queries_checked"], "mismatches": par["mismatches"], "checker": par["checker"],
        "distinct_batches_checked": par["distinct_batches_checked"]}
    line["latency_ms"] = None if lat is None else {"p50": round(lat["p50"], 4), "p99": round(lat["p99"], 4),
                                                   "n": lat["n"]}
    line["realloc_events_timed"] = out.get("realloc_events_timed")
    line["distinct_batches"] = out.get("distinct_batches")
    line["inflight"] = out.get("inflight")
    if out.get("legs"):
        line["legs"] = {name: _short_leg(leg) for name, leg in out["legs"].items()}
    if out.get("shard_transport"):
        t = out["shard_transport"]
        line["transport"] = t["transport"]
        line["rccl_ranks"] = t["rccl_ranks"]
    line["roofline_kernels"] = _short_kernels(out.get("roofline_kernels"))
    line["phase_ms"] = out.get("phase_ms")
    line["build"] = out.get("build")
    # the full record, written on the box that ran this (the driver's copy stays there;
    # everything the line's figures rest on is in the line itself)
    line["detail"] = detail
    return line


def transport_summary(infos):
    """One record for the line from every rank's yrwi_shard_info: the transport
    (one name when all ranks agree, else the per-rank list), RCCL communicator rank
    counts (min / max over the ranks), lanes with their own communicator, and the
    ranks that shared a device with another."""
    infos = [i for i in (infos or []) if i]
    if not infos:
        return None
    names = sorted({i["transport"] for i in infos})
    rr = [int(i["rccl_ranks"]) for i in infos]
    oc = [int(i["lanes_own_comm"]) for i in infos]
    return {"transport": names[0] if len(names) == 1 else [i["transport"] for i in infos],
            "rccl_ranks": {"min": min(rr), "max": max(rr)},
            "lanes_own_comm": {"min": min(oc), "max": max(oc)},
            "ranks": len(infos),
            "ranks_sharing_a_device": sum(1 for i in infos if int(i["device_peers"]) > 0),
            "pci_bus_ids": [i["pci_bus_id"] for i in infos]}


def _short_kernels(kern):
    """The per-kernel roofline block, a few fields per kernel (it is what the headline's
    roofline is chosen from)."""
    if not kern:
        return None
    keep = ("mean_launch_us", "achieved", "frac", "traffic", "hbm_frac", "rocprof_mean_launch_us")
    out = {}
    for name, r in kern.items():
        if isinstance(r, dict):
            out[name] = {k: (round(r[k], 4) if isinstance(r[k], float) else r[k]) for k in keep if r.get(k) is not None}
    return out


LEG_DESC = {
    "C3": "1B postings Zipf (100M URLs x 10k words), 1000 x 3-term AND + 1 excluded term, default profile, top-100",
    "C4": "4096 concurrent 2-4 term AND queries over the C3 index, default profile, top-100, one batch per step",
    "C5": "per-GPU slice (url-hash shards of the 8-way partition) of the 5B-posting corpus (500M URLs x 100k words), "
          "1000 x 2-4 term AND, custom profile date=15,domlength=15,authority=13,tf=10 and the /date profile",
}


def run_leg(R, leg, args, rank, world):
    """An extra BASELINE config on the same ranks: C3 / C4 strong-scale the fixed
    1B corpus over the N ranks; C5 gives every rank one 625M-posting url-hash shard
    of the 8-way partition of the 5B corpus.  On one GPU every leg also checks
    queries of its own timed batch against the oracle and times single queries."""
    from yacy_search_server_amd import RankingProfile, synth
    res = {}
    check = rank == 0 and world == 1
    nchk = 0 if args.no_cpu else args.leg_check
    nlat = args.leg_latency
    if leg in ("C3", "C4"):
        full = synth.preset("C3")
        cfg = full.shard(rank, world) if world > 1 else full
        if getattr(R, "leg_cfg", None) != ("C3", rank, world):
            R.close()
            R.leg_idx = None
            R.leg_idx, _ = R.open_index(cfg)
            R.leg_cfg = ("C3", rank, world)
        if leg == "C3":
            bats = draws(full, 1000, 3, 3, 1, None, args.batches)
        else:
            bats = draws(full, 4096, 2, 4, 0, full.seed ^ 0xC4, args.batches)
        hashes = [synth.term_hash(full, t) for t in range(full.n_terms)]
        prof = RankingProfile()
        M = R.measure(bats, hashes, prof, 100, args.leg_steps, 2 * args.inflight, args.inflight,
                      isolated=True)
        res[leg] = _leg_line(M, leg, len(bats[0]), world, "strong", load_pmc(leg) if world == 1 else None)
        if check:
            res[leg]["parity_sample"], res[leg]["latency_ms"] = check_and_latency(
                R, M, hashes, R.leg_idx, prof, 100, nchk, nlat, leg, threads=host_cores()[0])
    elif leg == "C5":
        full = synth.preset("C5")
        parts = max(8, world)
        R.close()
        R.leg_cfg = None
        R.leg_idx = None
        idx, _ = R.open_index(full.shard(rank, parts))
        bats = draws(full, 1000, 2, 4, 0, None, args.batches)
        hashes = [synth.term_hash(full, t) for t in range(full.n_terms)]
        custom = RankingProfile()
        custom.coeff_date, custom.coeff_domlength, custom.coeff_authority, custom.coeff_termfrequency = 15, 15, 13, 10
        for name, prof in (("C5_custom", custom), ("C5_date", RankingProfile.date())):
            M = R.measure(bats, hashes, prof, 100, args.leg_steps, 2 * args.inflight, args.inflight,
                          isolated=True)
            res[name] = _leg_line(M, "C5", len(bats[0]), world, "weak", load_pmc(name) if world == 1 else None)
            if check:
                res[name]["parity_sample"], res[name]["latency_ms"] = check_and_latency(
                    R, M, hashes, idx, prof, 100, nchk, nlat, name, threads=host_cores()[0])
        del idx
        R.close()
    else:
        raise ValueError(f"unknown leg {leg}")
    return res


def _leg_line(M, leg, nq, world, scaling, pmc=None):
    ms = M["dt"] / M["steps"] * 1e3
    roof, kern = roofline_block(M["iso"], M["timed"], M["steps"], ms, pmc)
    return {"workload": LEG_DESC[leg], "value": M["total_post"] / M["dt"], "unit": "postings/s", "n_gpus": world,
            "scaling": scaling, "steps": M["steps"], "ms_per_step": ms, "distinct_batches": M["D"],
            "identical_batch": M["identical"],
            "postings_per_step": M["total_post"] / M["steps"], "queries_per_step": nq,
            "roofline": roof, "roofline_kernels": kern, "joined_per_step": M["timed"]["joined"] / M["steps"],
            "realloc_events_timed": M["timed"]["n_realloc"], "phase_ms": phase_ms(M["iso"])}


def phase_ms(iso):
    """Per batch, from the library's own HIP events (isolated pass): join+probe
    kernels, compaction, normalisation (reduce..combine), scoring (score..emit),
    all kernels; host = call to results."""
    nbi = max(1, iso["batches"])
    return {"join": round(iso["t_join_ns"] / 1e6 / nbi, 3),
            "probe": round(iso["t_probe_ns"] / 1e6 / nbi, 3),
            "compact": round(iso["t_compact_ns"] / 1e6 / nbi, 3),
            "chain": round(iso.get("t_chain_ns", 0) / 1e6 / nbi, 3),
            "norm": round(iso["t_norm_ns"] / 1e6 / nbi, 3),
            "score": round(iso["t_score_ns"] / 1e6 / nbi, 3),
            "kernels": round(iso["t_kernels_ns"] / 1e6 / nbi, 3),
            "host_total": round(iso["t_total_ns"] / 1e6 / nbi, 3)}


def dry_run(args, rank, world):
    """Launcher check without a GPU: every rank joins a gloo group and rank 0 prints
    the JSON line's identity fields."""
    import torch
    import torch.distributed as tdist
    if world > 1:
        tdist.init_process_group("gloo")
        t = torch.tensor([rank + 1.0])
        tdist.all_reduce(t)
        tdist.barrier()
    if rank == 0:
        print(json.dumps({"metric": "postings joined+ranked/sec (node)", "dry_run": True, "n_gpus": world,
                          "ranks_sum": float(t.item()) if world > 1 else 1.0, "scaling": args.scaling,
                          "steps": args.steps, "warmup": args.warmup}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"--gpus {args.gpus} but WORLD_SIZE {world}: measuring {world} rank(s)")
    if args.dry_run:
        dry_run(args, rank, world)
        return
    run(args, rank, world, local)


if __name__ == "__main__":
    main()
