// yrwi_host.h -- host-side structures shared by libyrwi's host translation
// units (yrwi_host.cpp: contexts, planning, query execution; yrwi_heap.cpp:
// BLOB heap loader).  Internal; the public ABI is include/yrwi.h.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_set>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <map>
#include <unordered_map>
#include <numeric>
#include <string>
#include <vector>

#include "yrwi_internal.h"

namespace yrwi {

constexpr int64_t MAX_LIST = 53687091;  // RowSet.importRowSet: 2^31 bytes of 40-byte rows

// Base64Order.enhancedCoder alphabet index (Base64Order.java:38,54), -1 if not in it
struct AhpTable {
  int8_t v[256];
  constexpr AhpTable() : v() {
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    for (int i = 0; i < 256; i++) v[i] = -1;
    for (int i = 0; i < 64; i++) v[(uint8_t)a[i]] = (int8_t)i;
  }
};
inline constexpr AhpTable AHP_T{};
#define AHP AHP_T.v

struct KeyT {
  uint64_t hi;
  uint32_t lo;
  bool operator<(const KeyT& o) const { return hi < o.hi || (hi == o.hi && lo < o.lo); }
  bool operator==(const KeyT& o) const { return hi == o.hi && lo == o.lo; }
};

inline bool key_of(const uint8_t* h, KeyT* k) {
  uint64_t x = 0;
  for (int j = 0; j < 10; j++) {
    if (AHP[h[j]] < 0) return false;
    x = (x << 6) | (uint64_t)AHP[h[j]];
  }
  if (AHP[h[10]] < 0 || AHP[h[11]] < 0) return false;
  uint32_t c10 = (uint32_t)AHP[h[10]], c11 = (uint32_t)AHP[h[11]];
  k->hi = (x << 4) | (c10 >> 2);
  k->lo = ((c10 & 3u) << 6) | c11;
  return true;
}

// Java int arithmetic
inline int32_t add32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
inline int32_t mul32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
inline int log2j(int32_t x) {
  int l = 0;
  while (x > 0) { x >>= 1; l++; }
  return l;
}

struct ListRec {
  uint64_t* khi = nullptr;
  uint8_t* klo = nullptr;
  uint8_t* rows = nullptr;
  int64_t n = 0;
  uint32_t* uid = nullptr;  // url ids (rebuilt with the url dictionary)
  uint64_t* feat = nullptr; // ranking records (built with the url dictionary)
  uint32_t* head = nullptr; // line heads of uid (DList::head; rebuilt with the url ids)
  uint64_t* bm = nullptr;   // url-id bitmap (DList::bm; large lists only, rebuilt with the url ids)
  uint64_t* j5 = nullptr;   // record words 0-1 of the bitmap lists (DList::j5)
  DList dl() const { return DList{khi, klo, rows, n, uid, feat, head, nullptr, 0, bm, j5}; }
};

// device-wide allocation events (hipMalloc / hipFree / hipHostMalloc / hipHostFree
// on the query path: each one synchronises the whole device, so two lanes stop
// overlapping while it runs); reported per batch in yrwi_stats.n_realloc
inline std::atomic<int64_t> g_realloc{0};
inline thread_local int64_t t_realloc = 0;  // the calling thread's events (per-batch statistics)
// one device-wide allocation event (what and how much: the statistics count them)
inline void note_realloc(const char* what, size_t bytes) {
  (void)what;
  (void)bytes;
  g_realloc++;
  t_realloc++;
}

// bump allocator over device chunks
struct Arena {
  std::vector<std::pair<uint8_t*, size_t>> chunks;
  size_t used = 0, cur = 0, total_used = 0, min_chunk;
  explicit Arena(size_t mc) : min_chunk(mc) {}
  uint8_t* alloc(size_t bytes) {
    bytes = (bytes + 255) & ~(size_t)255;
    if (bytes == 0) bytes = 256;
    while (cur < chunks.size() && used + bytes > chunks[cur].second) {
      cur++;
      used = 0;
    }
    if (cur >= chunks.size()) {
      size_t sz = std::max(std::max(bytes, min_chunk), capacity());  // geometric: few hipMallocs
      note_realloc("arena grow", sz);
      void* p = nullptr;
      if (hipMalloc(&p, sz) != hipSuccess) return nullptr;
      chunks.push_back({(uint8_t*)p, sz});
      cur = chunks.size() - 1;
      used = 0;
    }
    uint8_t* p = chunks[cur].first + used;
    used += bytes;
    total_used += bytes;
    return p;
  }
  // only call when no kernel uses arena memory any more
  void reset() {
    if (chunks.size() > 1) {
      note_realloc("arena consolidate", total_used);
      size_t need = total_used + (1 << 20);
      for (auto& c : chunks) hipFree(c.first);
      chunks.clear();
      void* p = nullptr;
      if (hipMalloc(&p, std::max(need, min_chunk)) == hipSuccess)
        chunks.push_back({(uint8_t*)p, std::max(need, min_chunk)});
    }
    used = 0;
    cur = 0;
    total_used = 0;
  }
  // one chunk of at least `bytes` (no allocation in use: call between passes)
  void reserve(size_t bytes) {
    if (capacity() >= bytes && chunks.size() <= 1) return;
    note_realloc("arena reserve", bytes);
    for (auto& c : chunks) hipFree(c.first);
    chunks.clear();
    void* p = nullptr;
    if (hipMalloc(&p, std::max(bytes, min_chunk)) == hipSuccess) chunks.push_back({(uint8_t*)p, std::max(bytes, min_chunk)});
    used = cur = total_used = 0;
  }
  size_t capacity() const {
    size_t s = 0;
    for (auto& c : chunks) s += c.second;
    return s;
  }
  void release() {
    for (auto& c : chunks) hipFree(c.first);
    chunks.clear();
  }
};

struct Plan {
  bool empty = true;                 // no result anywhere (J1 on global sizes)
  std::vector<const ListRec*> seq;   // fold order; a list absent from this shard is an empty ListRec
  std::vector<int64_t> seq_ng;       // global size of each seq list (sum over shards)
  // include term i has a url-id bitmap on every shard (the planning exchange; one
  // context: its own list's): the count-first popcounts (cf3) are then shard-safe
  bool inc_allbm[YRWI_MAX_TERMS] = {};
  std::vector<const ListRec*> excl;  // this shard's exclusion lists (empty: no exclusion)
  // term keys (HandleSet order) and their lists on this shard (nullptr: absent)
  int ninc = 0, nexc = 0;
  KeyT inc[YRWI_MAX_TERMS], exc[YRWI_MAX_TERMS];
  const ListRec* linc[YRWI_MAX_TERMS];
  const ListRec* lexc[YRWI_MAX_TERMS];
  int32_t maxd = YRWI_MAX_DISTANCE_ANY, k = 0;
  yrwi_profile prof{};
  uint8_t lang[2] = {0, 0};
  int32_t lang_ok = 0;
  int64_t now_ms = 0;
  int64_t postings_in = 0;
  const yrwi_filter* filter = nullptr;  // addRWIs constraints (nullptr: none)
  // runtime container (a deferred one between the steps of a multi-term fold)
  DList cont{nullptr, nullptr, nullptr, 0};
  int32_t step_mode[YRWI_MAX_TERMS] = {0};  // JoinMode of every fold step taken
  // count-first chained fold (t = 3, list 2 the smallest): list 0 x list 1 only
  // counted (its size decides step 1's dispatch), the survivors chained from list 2
  bool cf = false;
  int64_t cf_count = 0;  // this shard's |list 0 x list 1|
  // from list 3 (t = 4, list 3 the smallest, lists 0..2 with bitmaps, one
  // context): |list 0 x list 1| and |list 0 x list 1 x list 2| both counted as
  // bitmap popcounts, the survivors chained from list 3
  bool cf3 = false;
  int64_t cf_count2 = 0;
  uint8_t* removed = nullptr;
  // normalisation pieces the last step's compaction wrote (JoinQ::psum): the rank
  // phase folds them instead of reading the container back (k_reduce), or nullptr
  const ChunkSum* pieces = nullptr;
  int64_t npieces = 0;
  int nexcl_g = 0;      // exclusion terms in effect (J1 on global sizes; excl holds this shard's lists of them)
  bool chain = false;   // chained fold (ChainQ, yrwi_internal.h): one join step, k_chain does the rest
  int seq_term[YRWI_MAX_TERMS] = {0};  // include term (linc index) of every seq list
  // TermSearch's urlselection (yrwi_query_desc.urlselection): its keys (sorted,
  // unique), their url ids on this shard (ascending; urls the dictionary does not
  // hold dropped), and the local sizes of the query's lists restricted to it
  bool has_sel = false;
  std::vector<KeyT> sel;
  std::vector<uint32_t> sel_uid;
  int64_t sel_ninc[YRWI_MAX_TERMS] = {0}, sel_nexc[YRWI_MAX_TERMS] = {0};
};


struct KeyHash {
  size_t operator()(const KeyT& k) const { return (size_t)(k.hi * 0x9E3779B97F4A7C15ull) ^ k.lo; }
};

// pinned host staging for the per-batch uploads (pageable copies would block)
struct Stage {
  uint8_t* p = nullptr;
  size_t cap = 0, used = 0;
};

// Pinned host buffers handed out by yrwi_host_alloc: results whose destination
// lies inside one are written there by the GPU directly (no staging copy).
struct HostRegistry {
  std::mutex mu;
  std::vector<std::pair<uint8_t*, size_t>> bufs;
  bool contains(const void* p, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu);
    const uint8_t* q = static_cast<const uint8_t*>(p);
    for (auto& b : bufs)
      if (q >= b.first && q + bytes <= b.first + b.second) return true;
    return false;
  }
};

struct LoopGroup;  // in-process shard group (yrwi_coll.cpp)
struct HostX;      // shared-memory mailbox of the node's ranks (yrwi_coll.cpp)
struct DevX;       // host-staged device collectives of the node's ranks (yrwi_coll.cpp)

// Order of the collectives of concurrently running batch parts (sharded
// contexts).  Every batch part gets a sequence number in
// submission order -- the same on every rank, since the ranks submit the same
// batches -- and may enqueue its collectives only once the part before it has
// enqueued its last one (CollTurn::next == its number).  So every rank enqueues
// all collectives in one total order, (part, step), whatever the timing of its
// lane threads: no rank can wait inside one communicator's collective for a
// peer that is blocked behind another's, even when both lanes' streams land on
// one hardware queue.
struct CollTurn {
  std::mutex mu;
  std::condition_variable cv;
  int64_t next = 0;
};

// One execution lane: a HIP stream with its own scratch arena, pinned staging,
// events and (sharded) communicator.  A batch is split over the lanes and each
// lane runs its part from its own host thread, so one lane's host planning and
// synchronisation overlap the other lane's kernels (and latency-bound kernels
// of the two lanes share the device).
struct Lane {
  int device = 0, rank = 0, world = 1;
  // the url-hash-shard protocol runs (global-size planning, collectives, shard
  // merge): world > 1, or a world-1 context over a real 1-rank RCCL communicator
  // (YRWI_COLL_SELF=1 at yrwi_open_shard: every RCCL call of the sharded path
  // runs with production counts, types and streams on one GPU)
  bool sharded = false;
  int nlanes = 1;  // lanes of the context (scratch budget share)
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  LoopGroup* loop = nullptr;  // test transport instead of comm (yrwi_coll.cpp)
  DevX* devx = nullptr;       // host-staged collectives instead of comm (RCCL could not form the group)
  int32_t dcall = 0;          // host-staged collective rounds of the running part
  hipEvent_t coll_ev[2] = {nullptr, nullptr};
  Stage stage;
  Stage out_stage;           // pinned landing buffer for results
  Stage down_stage;          // pinned landing buffer for small per-step readbacks (joined sizes)
  int64_t probe_ratio = 8;   // YRWI_PROBE_RATIO, read once per call
  bool band_order = true;    // band-major compaction schedule (BandOrder); YRWI_BAND_ORDER
  int64_t nurls = 0;         // url ids of the context's dictionary (set with dkhi)
  const uint64_t* dkhi = nullptr;  // the context's url dictionary keys (set when it is built)
  const uint8_t* dklo = nullptr;
  // the index records carry dense host ids (ensure_host_ids); host_key[id] = the host hash
  bool host_ids = false;
  const uint64_t* host_key = nullptr;
  Arena arena{(size_t)256 << 20};
  std::string err;
  std::vector<hipEvent_t> evpool;
  size_t evnext = 0;
  HostRegistry* hostreg = nullptr;
  hipEvent_t sync_ev = nullptr;
  bool own_stream = true;
  // persistent worker thread; `done` = last finished async ticket
  int64_t done = -1;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;
  bool busy = false, quit = false;
  // active: a batch runs on this lane (worker or calling thread); reserving:
  // another lane's thread is sizing this lane's arena (see share_arena_size)
  bool active = false, reserving = false;
  int rc = 0;
  int64_t wait_ns = 0;  // host time spent waiting for this lane's device work (lane_sync)
  // scratch high-water mark of the context's lanes (bytes): a lane whose arena is
  // smaller takes that size at the start of its next pass instead of growing
  // inside it (one allocation, before any of the pass's kernels)
  std::atomic<size_t>* scratch_hint = nullptr;
  // the scratch the lanes may use together (bytes; 0: not measured yet): device
  // memory left after the index, dictionary and bitmaps (ensure_url_ids)
  std::atomic<int64_t>* scratch_total = nullptr;
  // collective order (CollTurn): the running part's sequence number (-1: none,
  // unordered), whether it holds the turn, and whether its last pass passes the
  // turn on right after its final collective
  CollTurn* turn = nullptr;
  int64_t seq = -1;
  HostX* hostx = nullptr;  // host exchange of the batch part's list sizes (shared by the lanes)
  int32_t xcall = 0;       // exchanges made by the running part
  bool turn_held = false, release_after_final = false;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  hipEvent_t event() {
    if (evnext >= evpool.size()) {
      hipEvent_t e;
      hipEventCreate(&e);
      evpool.push_back(e);
    }
    return evpool[evnext++];
  }
  void start_worker() {
    th = std::thread([this] {
      hipSetDevice(device);
      std::unique_lock<std::mutex> lk(mu);
      while (true) {
        cv.wait(lk, [this] { return busy || quit; });
        if (quit) return;
        lk.unlock();
        job();
        lk.lock();
        busy = false;
        cv.notify_all();
      }
    });
  }
  void submit(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu);
    job = std::move(f);
    busy = true;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return !busy && !reserving; });
  }
  void enter() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return !reserving; });
    active = true;
  }
  void leave() {
    std::lock_guard<std::mutex> lk(mu);
    active = false;
    cv.notify_all();
  }
  // size this (idle) lane's arena from another thread; false if the lane is in use
  bool try_reserve(size_t bytes) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (busy || active || reserving) return false;
      reserving = true;
    }
    arena.reserve(bytes);
    std::lock_guard<std::mutex> lk(mu);
    reserving = false;
    cv.notify_all();
    return true;
  }
  void stop() {
    if (!th.joinable()) return;
    {
      std::lock_guard<std::mutex> lk(mu);
      quit = true;
      cv.notify_all();
    }
    th.join();
  }
};

struct CtxBase {
  int device = 0, rank = 0, world = 1;
  bool sharded = false;  // Lane::sharded
  hipStream_t stream = nullptr;  // == lanes[0]->stream (index uploads)
  std::vector<Lane*> lanes;
  HostRegistry hostreg;
  // asynchronous batches: ticket t runs on lane t % lanes; finished status by ticket
  int64_t next_ticket = 0;
  // collective order of batch parts (sequence numbers handed out by the caller's thread)
  CollTurn turn;
  int64_t coll_seq = 0;
  HostX* hostx = nullptr;
  DevX* devx = nullptr;
  int transport = 0;  // YRWI_TRANSPORT_* (yrwi_shard_info): how the shards' collectives travel
  int device_peers = -1;  // other ranks of the group on this device (-1: unknown / not exchanged)
  std::atomic<size_t> scratch_hint{0};  // Lane::scratch_hint
  std::atomic<int64_t> scratch_total{0};  // Lane::scratch_total
  std::mutex st_mu;
  std::unordered_map<int64_t, std::pair<int, std::string>> status;
  std::unordered_map<KeyT, ListRec, KeyHash> lists;
  Arena index_mem{(size_t)1 << 30};
  // url dictionary (yrwi_dict.hip): every list's uid array is a slice of uid_all;
  // rebuilt before the next query after any list changed
  bool uid_dirty = true;
  uint32_t* uid_all = nullptr;   // list slices start on 128-B lines (32 ids)
  size_t uid_cap = 0;
  uint32_t* head_all = nullptr;  // every list's line heads (DList::head)
  size_t head_cap = 0;
  uint64_t* bm_all = nullptr;    // the bitmaps of the large lists (DList::bm)
  size_t bm_cap = 0;
  uint64_t* dkhi = nullptr;  // key of every url id (72-bit Base64 key: hi 64 bits, low byte)
  uint8_t* dklo = nullptr;
  size_t dict_cap = 0;
  int64_t nurls = 0;
  // dense host ids (authority host counts, yrwi_dict.hip ensure_host_ids): every
  // index record carries its url's host id; host_key[id] = the host hash (url-hash
  // chars 6..11, 36 bits).  Built on the first authority batch after an index
  // change, dropped by any change.
  bool host_ids = false;
  uint64_t* host_key = nullptr;
  size_t host_key_cap = 0;
  int64_t nhosts = 0;
  // incremental maintenance (yrwi_dict.hip): lists added or replaced since the
  // dictionary was last brought up to date; keys of removed postings stay in it
  // (an id without postings changes no join) until the next full rebuild
  std::unordered_set<KeyT, KeyHash> dict_pending;
  bool dict_valid = false;   // every list outside dict_pending has url ids in the dictionary
  int64_t dict_churn = 0;    // postings removed or replaced since the last full rebuild
  int64_t index_repacks = 0; // index memory compactions (yrwi_dict.hip repack_index)
  size_t repack_blocked_at = SIZE_MAX;  // index_mem.total_used when a repack last failed (not retried until it changes)
  int64_t dict_full_builds = 0, dict_incremental = 0;
  std::string err;
  int64_t npostings = 0;
  // search events (yrwi_event.cpp): their entry points serialise on api_mu; device
  // blocks of closed order-only events are reused (bytes, pointer)
  std::recursive_mutex api_mu;
  std::mutex ev_pool_mu;
  std::vector<std::pair<size_t, void*>> ev_pool;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  // a lane's error becomes the context's
  int take(Lane* l, int rc) {
    if (rc) err = l->err;
    return rc;
  }
};

void drain(CtxBase* ctx);
// yrwi_filter -> FilterQ (device pointers unset) + sorted unique siteexclude host keys and doublecheck url keys
void build_filterq(const yrwi_filter& F, FilterQ* G, std::vector<uint64_t>* siteex, std::vector<KeyT>* urls);

#define HIPCHK(ctx, x)                                                                 \
  do {                                                                                \
    hipError_t _e = (x);                                                              \
    if (_e != hipSuccess) return (ctx)->fail(YRWI_E_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

template <class T>
inline T* arena_alloc(Lane* ctx, int64_t count) {
  return reinterpret_cast<T*>(ctx->arena.alloc((size_t)std::max<int64_t>(count, 1) * sizeof(T)));
}

// Wait for this lane's work so far: an event, not a stream sync, so lanes that
// share one stream do not wait for work the other lane enqueues later.
inline hipError_t lane_sync(Lane* L) {
  // (a blocking-sync event or a polled wait, measured in round 2: no better,
  // profiles/archive/r02f_sync_poll_sweep.txt)
  if (!L->sync_ev && hipEventCreateWithFlags(&L->sync_ev, hipEventDisableTiming) != hipSuccess)
    return hipErrorOutOfMemory;
  hipError_t e = hipEventRecord(L->sync_ev, L->stream);
  if (e != hipSuccess) return e;
  const auto t0 = std::chrono::steady_clock::now();
  e = hipEventSynchronize(L->sync_ev);
  L->wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  return e;
}

// pinned buffer of at least `bytes` (contents dropped on growth); nullptr on failure
inline uint8_t* stage_reserve(Lane* ctx, Stage* S, size_t bytes, bool drain) {
  if (bytes > S->cap) {
    note_realloc("pinned stage", bytes);
    if (drain && lane_sync(ctx) != hipSuccess) return nullptr;
    if (S->p) hipHostFree(S->p);
    S->p = nullptr;
    S->cap = std::max<size_t>(std::max<size_t>(2 * S->cap, bytes), (size_t)4 << 20);
    if (hipHostMalloc(reinterpret_cast<void**>(&S->p), S->cap, hipHostMallocDefault) != hipSuccess) {
      S->cap = 0;
      ctx->fail(YRWI_E_HIP, "pinned host allocation failed");
      return nullptr;
    }
  }
  return S->p;
}

// Host -> device uploads of per-batch descriptors.  The bytes are staged in the
// lane's pinned buffer and pulled by ONE copy kernel per call (k_copy_in reads
// the pinned pages through their device address) on the lane's stream: no DMA
// engine on the query path.  SDMA copies measured 1.3-1.5 ms per C2 batch over
// the driver's 20-step run against 0.8 with HSA_ENABLE_SDMA=0 (the copy engines'
// queues stall the lanes' first batches: profiles/archive/r03a_sdma.txt).
struct UpEnt {
  void* dst;
  const void* src;
  size_t bytes;
};

inline int upload_list(Lane* ctx, const UpEnt* e, int n) {
  Stage& S = ctx->stage;
  size_t need = S.used;
  for (int i = 0; i < n; i++) need = ((need + 255) & ~(size_t)255) + e[i].bytes;
  if (need > S.cap) {
    note_realloc("pinned upload stage", need);
    // copy kernels still read the old buffer: drain them, then grow
    HIPCHK(ctx, lane_sync(ctx));
    if (S.p) HIPCHK(ctx, hipHostFree(S.p));
    S.p = nullptr;
    S.cap = std::max<size_t>(std::max<size_t>(2 * S.cap, need - S.used + 256 * (size_t)n), (size_t)4 << 20);
    HIPCHK(ctx, hipHostMalloc(reinterpret_cast<void**>(&S.p), S.cap, hipHostMallocDefault));
    S.used = 0;
  }
  uint8_t* d_base = nullptr;
  HIPCHK(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&d_base), S.p, 0));
  CopyIn c{};
  for (int i = 0; i < n; i++) {
    if (e[i].bytes == 0) continue;
    const size_t off = (S.used + 255) & ~(size_t)255;
    std::memcpy(S.p + off, e[i].src, e[i].bytes);
    S.used = off + e[i].bytes;
    if (c.n == COPY_IN_MAX) {
      if (launch_copy_in(c, ctx->stream)) return ctx->fail(YRWI_E_HIP, "copy-in launch");
      c = CopyIn{};
    }
    c.src[c.n] = d_base + off;
    c.dst[c.n] = static_cast<uint8_t*>(e[i].dst);
    c.bytes[c.n] = e[i].bytes;
    c.n++;
  }
  if (c.n && launch_copy_in(c, ctx->stream)) return ctx->fail(YRWI_E_HIP, "copy-in launch");
  return 0;
}

inline void up_collect(UpEnt*, int&) {}
template <class T, class... R>
inline void up_collect(UpEnt* e, int& n, T* dst, const std::vector<T>& v, R&&... rest) {
  e[n++] = UpEnt{dst, v.data(), v.size() * sizeof(T)};
  up_collect(e, n, std::forward<R>(rest)...);
}

// upload(ctx, d_a, va, d_b, vb, ...): every (device destination, host vector)
// pair in one copy kernel
template <class T, class... R>
inline int upload(Lane* ctx, T* dst, const std::vector<T>& v, R&&... rest) {
  UpEnt e[1 + sizeof...(R) / 2];
  int n = 0;
  up_collect(e, n, dst, v, std::forward<R>(rest)...);
  return upload_list(ctx, e, n);
}

// Device -> host readback by a kernel writing the lane's pinned staging S (no
// copy engine on the query path): n elements of `elem` bytes, `stride` bytes
// apart in device memory.  Returns the host address of the packed result, valid
// after the next lane_sync; nullptr on failure.  One readback per stage at a time.
inline uint8_t* readback(Lane* L, Stage* S, const void* d_src, int64_t n, int32_t elem, int64_t stride) {
  uint8_t* h = stage_reserve(L, S, (size_t)std::max<int64_t>(n, 1) * elem, true);
  if (!h) return nullptr;
  uint8_t* d = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess ||
      launch_gather_out(d, static_cast<const uint8_t*>(d_src), n, elem, stride, L->stream)) {
    L->fail(YRWI_E_HIP, "readback launch");
    return nullptr;
  }
  return h;
}

// start of a device pass: nothing is in flight any more, scratch can be reused
inline int begin_pass(Lane* ctx) {
  HIPCHK(ctx, lane_sync(ctx));
  ctx->arena.reset();
  if (ctx->scratch_hint) {
    const size_t h = ctx->scratch_hint->load();
    if (ctx->arena.capacity() < h) ctx->arena.reserve(h);
  }
  ctx->stage.used = 0;
  ctx->evnext = 0;
  const char* e = getenv("YRWI_PROBE_RATIO");  // tests force either join algorithm with it
  ctx->probe_ratio = e ? std::max<int64_t>(1, atoll(e)) : (int64_t)8;
  const char* b = getenv("YRWI_BAND_ORDER");  // 0: job-order tile schedule (A/B measurements; same results)
  ctx->band_order = !(b && b[0] == '0');
  return 0;
}

// ---- collectives between url-hash shards (yrwi_coll.cpp): RCCL over xGMI, or
// the in-process loopback group that lets tests run several shards on one GPU.
struct Xfer {
  int peer;
  void* ptr;
  size_t bytes;
};
// (re)build the url dictionary and every list's url ids if the index changed
int ensure_url_ids(CtxBase* ctx);
// device memory left for the lanes' scratch after the index is resident (CtxBase::scratch_total)
void measure_scratch(CtxBase* ctx);
// dense host ids in every index record (after ensure_url_ids; no batch in flight)
int ensure_host_ids(CtxBase* ctx);
// the list of `term` was added / replaced (added = true) or removed: url ids are due
void index_changed(CtxBase* ctx, const KeyT& term, int64_t old_n, bool added);
// brings the url ids up to date, then counts inconsistencies (0: every id names its key)
int check_url_ids(CtxBase* ctx, int64_t* bad);

HostX* hostx_open(const uint8_t id[128], int world, int rank);  // nullptr: not available (device fallback)
void hostx_close(HostX* x, bool unlink_name);
void hostx_abort(HostX* x, int64_t seq);  // batch part `seq` failed: every rank's exchanges of that part fail at once
int hostx_attached(const HostX* x);  // ranks that mapped the segment so far (0: no mailbox)
bool hostx_wait_attached(const HostX* x, double limit_s);  // every rank mapped it (false: timeout)
// other ranks of the group on this rank's device (-1: some rank never posted its identity)
int hostx_device_peers(const HostX* x, int64_t my_devid, double limit_s);
int hostx_allsum(Lane* L, std::vector<int64_t>& v);  // 0 done, 1 not handled, < 0 error
// host-staged device collectives (ranks that share a device: RCCL refuses them)
DevX* devx_open(const uint8_t id[128], int world, int rank, HostX* hx);
void devx_close(DevX* x, bool unlink_name);
void turn_acquire(Lane* L);  // wait until L's batch part may enqueue collectives (no-op: seq < 0)
void turn_release(Lane* L);  // pass the turn to the next part (waits for L's turn first); idempotent
int coll_allgather(Lane* L, const void* send, void* recv, size_t bytes);  // recv: world * bytes, rank order
int coll_allreduce_i32(Lane* L, int32_t* buf, size_t n, bool max_op);    // in place; sum or max
int coll_exchange(Lane* L, const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs);  // grouped send/recv
// loopback groups: a 128-byte id starting with this tag names an in-process group
constexpr char LOOP_TAG[] = "YRWI-LOOPBACK";
// a 128-byte id starting with this tag names a group of processes that share one
// device: host-staged collectives without trying RCCL first
constexpr char STAGE_TAG[] = "YRWI-HOSTSTAGE";
LoopGroup* loop_join(const uint8_t id[128], int world, int rank);
void loop_leave(LoopGroup* g);

}  // namespace yrwi

// the opaque context of the C ABI
struct yrwi_ctx : yrwi::CtxBase {};
