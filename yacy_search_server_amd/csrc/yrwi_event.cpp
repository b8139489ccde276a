// yrwi_event.cpp -- search events: one SearchEvent's RWI side receiving
// containers one after another.  The local joined
// container and every remote peer's result container go through
// SearchEvent.addRWIs (SearchEvent.java:673-836; remote: Protocol.java:802) and
// the event's ReferenceOrder, doublecheck set, flag counts and rwiStack carry
// over between arrivals.  All of that state lives in device memory; k_event_add
// (yrwi_kernels.hip) applies a batch of arrivals, one workgroup per event.
#include <map>

#include "yrwi_host.h"

using namespace yrwi;

// One doubleDomCache queue entry (SearchEvent.java:1319-1339): a polled stack entry
// and when it was queued (the tie-break between equal heads of different hosts).
struct DDEntry {
  yrwi_hit h;
  uint64_t seq;
};

struct yrwi_event {
  EvDev h{};         // host copy of the device descriptor
  void* mem = nullptr;
  size_t bytes = 0;  // of mem
  bool pooled = false;  // order-only event: mem goes back to the context's pool at close
  int32_t k = 0;
  // SearchEvent.doubleDomCache: host hash (url-hash chars 6..11) -> that host's
  // queued entries in ReverseElement order; a host with an empty queue has had
  // one entry returned and none queued since
  std::map<uint64_t, std::vector<DDEntry>> dd;
  uint64_t dd_next = 0;
  // order-only authority events: an upper bound of the distinct hosts in the host
  // table (postings given since the last exact count); the table grows before a
  // container could fill it (grow_host_table)
  int64_t hosts_bound = 0;
};

namespace {

int ceil_log2(int64_t x) {
  int l = 0;
  while ((int64_t(1) << l) < x) l++;
  return l;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// the kernels' host-table hash (yrwi_kernels.hip mix64), for rehashing on the host
uint64_t mix64_host(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// order-only event block: state, host keys, host counts
struct OrderLayout {
  size_t o_hk, o_hc, need;
  explicit OrderLayout(int64_t hslots) {
    o_hk = align256(sizeof(EvState));
    o_hc = o_hk + align256((size_t)hslots * 8);
    need = o_hc + align256((size_t)hslots * 4);
  }
};

}  // namespace

// the event entry points may be called from several host threads (YaCy scores
// remote peers' containers on their own threads): one at a time per context
#define EVENT_LOCK(ctx) std::lock_guard<std::recursive_mutex> _evlk((ctx)->api_mu)

static void fill_rankq(RankQ& q, const yrwi_profile* prof, const char* language, int64_t now_ms) {
  if (prof) q.prof = *prof; else yrwi_profile_default(&q.prof);
  const char* lang = language ? language : "";
  const size_t ll = std::strlen(lang);
  q.lang_ok = ll == 2;
  q.lang[0] = ll > 0 ? (uint8_t)lang[0] : 0;
  q.lang[1] = ll > 1 ? (uint8_t)lang[1] : 0;
  q.now_ms = now_ms != 0 ? now_ms
                         : (int64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
                               std::chrono::system_clock::now().time_since_epoch()).count();
  q.want_authority = q.prof.coeff_authority > 12;
}

extern "C" int yrwi_event_open_order(yrwi_ctx* ctx, const yrwi_profile* prof, const char* language, int64_t now_ms,
                                     int64_t max_hosts, yrwi_event** out) {
  if (!ctx || !out || max_hosts < 0) return YRWI_E_ARG;
  *out = nullptr;
  EVENT_LOCK(ctx);
  hipSetDevice(ctx->device);
  EvDev h{};
  RankQ& q = h.q;
  fill_rankq(q, prof, language, now_ms);
  q.k = 1;
  // no url set, no stack (yrwi_event_order touches neither): the state and, for an
  // authority profile, the host table (2 slots per expected host)
  const int64_t hslots = q.want_authority ? (int64_t)1 << ceil_log2(std::max<int64_t>(2 * max_hosts, 64)) : 1;
  q.hmask = (uint64_t)(hslots - 1);
  const OrderLayout lay(hslots);
  const size_t o_st = 0, o_hk = lay.o_hk, o_hc = lay.o_hc, need = lay.need;
  // device memory from the context's pool of closed order-only events (a hipMalloc
  // would synchronise the whole device once per SearchEvent)
  void* mem = nullptr;
  size_t bytes = 0;
  {
    std::lock_guard<std::mutex> lk(ctx->ev_pool_mu);
    for (size_t i = 0; i < ctx->ev_pool.size(); i++)
      if (ctx->ev_pool[i].first >= need && ctx->ev_pool[i].first <= 4 * need + (1 << 20)) {
        bytes = ctx->ev_pool[i].first;
        mem = ctx->ev_pool[i].second;
        ctx->ev_pool.erase(ctx->ev_pool.begin() + (std::ptrdiff_t)i);
        break;
      }
  }
  if (!mem) {
    if (hipMalloc(&mem, need) != hipSuccess) return ctx->fail(YRWI_E_NOMEM, "event allocation failed");
    bytes = need;
  }
  uint8_t* base = static_cast<uint8_t*>(mem);
  h.st = reinterpret_cast<EvState*>(base + o_st);
  q.hkeys = reinterpret_cast<uint64_t*>(base + o_hk);
  q.hcnt = reinterpret_cast<uint32_t*>(base + o_hc);
  // zeroed on the order lane's stream, which runs every later call of the event
  Lane* L = ctx->lanes[0];
  if (hipMemsetAsync(base, 0, need, L->stream) != hipSuccess) {
    std::lock_guard<std::mutex> lk(ctx->ev_pool_mu);
    ctx->ev_pool.emplace_back(bytes, mem);
    return ctx->fail(YRWI_E_HIP, "event init");
  }
  yrwi_event* e = new yrwi_event;
  e->h = h;
  e->mem = mem;
  e->bytes = bytes;
  e->pooled = true;
  e->k = 1;
  *out = e;
  return 0;
}

extern "C" int yrwi_event_open(yrwi_ctx* ctx, const yrwi_profile* prof, const char* language, int64_t now_ms,
                               int32_t k, const yrwi_filter* filter, int64_t max_postings, yrwi_event** out) {
  if (!ctx || !out || k <= 0 || k > YRWI_MAX_K || max_postings < 0) return YRWI_E_ARG;
  *out = nullptr;
  EVENT_LOCK(ctx);
  if (filter && (filter->nsiteexcludes < 0 || filter->nurlhashes < 0 ||
                 (filter->nsiteexcludes > 0 && !filter->siteexcludes) || (filter->nurlhashes > 0 && !filter->urlhashes)))
    return ctx->fail(YRWI_E_ARG, "filter: bad siteexcludes / urlhashes");
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);

  EvDev h{};
  RankQ& q = h.q;
  fill_rankq(q, prof, language, now_ms);
  q.k = k;
  std::vector<uint64_t> siteex;
  std::vector<KeyT> seeds;
  if (filter) {
    build_filterq(*filter, &h.f, &siteex, &seeds);
    h.f.nurl = 0;  // the doublecheck seeds go into the url set
    h.f.flagcount = nullptr;
    h.has_filter = 1;
  }
  // url set: EV_SUBS sub-tables, each about 4x its share of the keys
  const int64_t cap = std::max<int64_t>(max_postings + (int64_t)seeds.size(), 1024);
  h.ulog = std::max(5, ceil_log2((4 * cap + EV_SUBS - 1) / EV_SUBS));
  const int64_t uslots = (int64_t)EV_SUBS << h.ulog;
  const int64_t hslots = q.want_authority ? (int64_t)1 << ceil_log2(2 * cap) : 1;
  q.hmask = (uint64_t)(hslots - 1);

  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align256(bytes);
    return o;
  };
  const size_t o_st = take(sizeof(EvState));
  const size_t o_uk = take((size_t)uslots * 8), o_uv = take((size_t)uslots * 8);
  const size_t o_hk = take((size_t)hslots * 8), o_hc = take((size_t)hslots * 4);
  const size_t o_stk = take((size_t)2 * k * sizeof(yrwi_hit));
  const size_t o_sx = take(std::max<size_t>(siteex.size(), 1) * 8);
  const size_t o_dev = take(sizeof(EvDev));
  const size_t o_sh = take(std::max<size_t>(seeds.size(), 1) * 8), o_sl = take(std::max<size_t>(seeds.size(), 1));
  void* mem = nullptr;
  if (hipMalloc(&mem, off) != hipSuccess) return ctx->fail(YRWI_E_NOMEM, "event allocation failed");
  uint8_t* base = static_cast<uint8_t*>(mem);
  h.st = reinterpret_cast<EvState*>(base + o_st);
  h.ukey = reinterpret_cast<uint64_t*>(base + o_uk);
  h.uval = reinterpret_cast<uint64_t*>(base + o_uv);
  q.hkeys = reinterpret_cast<uint64_t*>(base + o_hk);
  q.hcnt = reinterpret_cast<uint32_t*>(base + o_hc);
  h.stack = reinterpret_cast<yrwi_hit*>(base + o_stk);
  h.f.siteex = reinterpret_cast<uint64_t*>(base + o_sx);
  EvDev* d_dev = reinterpret_cast<EvDev*>(base + o_dev);

  auto fail = [&](int code, const char* m) {
    lane_sync(L);
    hipFree(mem);
    return ctx->fail(code, m);
  };
  hipStream_t s = L->stream;
  if (hipMemsetAsync(base, 0, off, s) != hipSuccess || hipMemsetAsync(h.uval, 0xFF, (size_t)uslots * 8, s) != hipSuccess)
    return fail(YRWI_E_HIP, "event init");
  std::vector<uint64_t> sh;
  std::vector<uint8_t> sl;
  for (auto& key : seeds) {
    sh.push_back(key.hi);
    sl.push_back((uint8_t)key.lo);
  }
  std::vector<EvDev> hv{h};
  if (upload(L, reinterpret_cast<uint64_t*>(base + o_sx), siteex, d_dev, hv, reinterpret_cast<uint64_t*>(base + o_sh), sh, base + o_sl, sl))
    return fail(YRWI_E_HIP, "event upload");
  if (launch_event_seed(d_dev, reinterpret_cast<uint64_t*>(base + o_sh), base + o_sl, (int64_t)sh.size(), s))
    return fail(YRWI_E_HIP, "event seed launch");
  int32_t err = 0;
  if (hipMemcpyAsync(&err, &h.st->err, 4, hipMemcpyDeviceToHost, s) != hipSuccess || lane_sync(L) != hipSuccess)
    return fail(YRWI_E_HIP, "event open sync");
  if (err) return fail(err, "doublecheck seeds exceed the event's url table");
  yrwi_event* e = new yrwi_event;
  e->h = h;
  e->mem = mem;
  e->bytes = off;
  e->k = k;
  *out = e;
  return 0;
}

extern "C" int yrwi_event_add(yrwi_ctx* ctx, yrwi_arrival* arr, int32_t narr) {
  if (!ctx || narr < 0 || (narr > 0 && !arr)) return YRWI_E_ARG;
  EVENT_LOCK(ctx);
  if (narr == 0) return 0;
  for (int32_t i = 0; i < narr; i++) {
    arr[i].rc = 0;
    if (!arr[i].ev || arr[i].n < 0 || arr[i].n >= ((int64_t)1 << 31) || (arr[i].n > 0 && !arr[i].rows40))
      return ctx->fail(YRWI_E_ARG, "bad arrival");
  }
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  // group the arrivals by event (first-appearance order), keeping their order inside a group
  std::unordered_map<const yrwi_event*, int32_t> gid;
  std::vector<const yrwi_event*> evs;
  for (int32_t i = 0; i < narr; i++)
    if (gid.emplace(arr[i].ev, (int32_t)evs.size()).second) evs.push_back(arr[i].ev);
  std::vector<std::vector<int32_t>> members(evs.size());
  for (int32_t i = 0; i < narr; i++) members[(size_t)gid[arr[i].ev]].push_back(i);
  int64_t total = 0;
  for (int32_t i = 0; i < narr; i++) total += arr[i].n;
  uint8_t* d_rows = arena_alloc<uint8_t>(L, total * YRWI_ROW_BYTES);
  EvDev* d_ev = arena_alloc<EvDev>(L, (int64_t)evs.size());
  EvJob* d_jobs = arena_alloc<EvJob>(L, narr);
  int32_t* d_jb = arena_alloc<int32_t>(L, (int64_t)evs.size() + 1);
  int32_t* d_status = arena_alloc<int32_t>(L, narr);
  if (!d_rows || !d_ev || !d_jobs || !d_jb || !d_status) return ctx->fail(YRWI_E_NOMEM, "arena");
  // the rows of every arrival, concatenated through pinned staging
  uint8_t* stg = stage_reserve(L, &L->out_stage, (size_t)std::max<int64_t>(total * YRWI_ROW_BYTES, 4), true);
  if (!stg) return ctx->take(L, YRWI_E_HIP);
  std::vector<EvDev> hev;
  std::vector<EvJob> jobs;
  std::vector<int32_t> jb{0}, job_arr;
  int64_t roff = 0;
  for (size_t g = 0; g < evs.size(); g++) {
    hev.push_back(evs[g]->h);
    for (int32_t i : members[g]) {
      EvJob J{};
      J.ev = (int32_t)g;
      J.local = arr[i].local != 0;
      J.rows = d_rows + roff * YRWI_ROW_BYTES;
      J.n = arr[i].n;
      if (arr[i].n) std::memcpy(stg + roff * YRWI_ROW_BYTES, arr[i].rows40, (size_t)arr[i].n * YRWI_ROW_BYTES);
      roff += arr[i].n;
      jobs.push_back(J);
      job_arr.push_back(i);
    }
    jb.push_back((int32_t)jobs.size());
  }
  hipStream_t s = L->stream;
  if (total) HIPCHK(ctx, hipMemcpyAsync(d_rows, stg, (size_t)total * YRWI_ROW_BYTES, hipMemcpyHostToDevice, s));
  if (upload(L, d_ev, hev, d_jobs, jobs, d_jb, jb)) return ctx->take(L, YRWI_E_HIP);
  if (launch_event_add(d_ev, d_jobs, d_jb, (int32_t)evs.size(), d_status, s))
    return ctx->fail(YRWI_E_HIP, "event_add launch");
  std::vector<int32_t> st((size_t)narr);
  HIPCHK(ctx, hipMemcpyAsync(st.data(), d_status, (size_t)narr * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(ctx, lane_sync(L));
  int first = 0;
  for (size_t j = 0; j < job_arr.size(); j++) {
    arr[job_arr[j]].rc = st[j];
    if (st[j] && !first) first = st[j];
  }
  if (first == YRWI_E_HASH) return ctx->fail(first, "arrival: url hash is not well-formed Base64");
  if (first == YRWI_E_NULL_LANGUAGE) return ctx->fail(first, "arrival: row with empty language cell (reference NPE)");
  if (first == YRWI_E_CAPACITY) return ctx->fail(first, "event tables full: max_postings too small");
  return first;
}

// ReferenceOrder.doms is an unbounded map (ReferenceOrder.java:176-198): an
// order-only event's host table (sized by the caller's expected hosts) grows
// before a container of `incoming` postings could fill it past 3/4 -- the live
// hosts are counted exactly when the running bound says it might, and rehashed
// into a table twice their (count + incoming) on the host (rare: the table at
// least doubles each time).  The state moves to the new block as it is.
static int grow_host_table(yrwi_ctx* ctx, yrwi_event* ev, int64_t incoming) {
  RankQ& q = ev->h.q;
  if (!q.want_authority || !ev->pooled) return 0;
  const int64_t slots = (int64_t)q.hmask + 1;
  if (ev->hosts_bound + incoming <= slots / 4 * 3) return 0;
  Lane* L = ctx->lanes[0];
  std::vector<uint64_t> keys((size_t)slots);
  std::vector<uint32_t> cnt((size_t)slots);
  HIPCHK(ctx, hipMemcpyAsync(keys.data(), q.hkeys, (size_t)slots * 8, hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, hipMemcpyAsync(cnt.data(), q.hcnt, (size_t)slots * 4, hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, lane_sync(L));
  int64_t used = 0;
  for (uint64_t k : keys) used += k != 0;
  ev->hosts_bound = used;
  if (used + incoming <= slots / 4 * 3) return 0;
  const int64_t ns = (int64_t)1 << ceil_log2(std::max<int64_t>(2 * (used + incoming), 2 * slots));
  const OrderLayout lay(ns);
  std::vector<uint64_t> nk((size_t)ns, 0);
  std::vector<uint32_t> nc((size_t)ns, 0);
  for (int64_t i = 0; i < slots; i++) {
    if (!keys[(size_t)i]) continue;
    uint64_t t = mix64_host(keys[(size_t)i]) & (uint64_t)(ns - 1);
    while (nk[(size_t)t]) t = (t + 1) & (uint64_t)(ns - 1);
    nk[(size_t)t] = keys[(size_t)i];
    nc[(size_t)t] = cnt[(size_t)i];
  }
  void* mem = nullptr;
  if (hipMalloc(&mem, lay.need) != hipSuccess) return ctx->fail(YRWI_E_NOMEM, "event host table growth");
  uint8_t* base = static_cast<uint8_t*>(mem);
  auto* nst = reinterpret_cast<EvState*>(base);
  auto* nhk = reinterpret_cast<uint64_t*>(base + lay.o_hk);
  auto* nhc = reinterpret_cast<uint32_t*>(base + lay.o_hc);
  if (hipMemcpyAsync(nst, ev->h.st, sizeof(EvState), hipMemcpyDeviceToDevice, L->stream) != hipSuccess ||
      hipMemcpyAsync(nhk, nk.data(), (size_t)ns * 8, hipMemcpyHostToDevice, L->stream) != hipSuccess ||
      hipMemcpyAsync(nhc, nc.data(), (size_t)ns * 4, hipMemcpyHostToDevice, L->stream) != hipSuccess ||
      lane_sync(L) != hipSuccess) {
    hipFree(mem);
    return ctx->fail(YRWI_E_HIP, "event host table growth copy");
  }
  {
    std::lock_guard<std::mutex> lk(ctx->ev_pool_mu);
    if (ctx->ev_pool.size() < 64) {
      ctx->ev_pool.emplace_back(ev->bytes, ev->mem);
      ev->mem = nullptr;
    }
  }
  if (ev->mem) hipFree(ev->mem);
  ev->mem = mem;
  ev->bytes = lay.need;
  ev->h.st = nst;
  q.hkeys = nhk;
  q.hcnt = nhc;
  q.hmask = (uint64_t)(ns - 1);
  return 0;
}

extern "C" int yrwi_event_order(yrwi_ctx* ctx, yrwi_event* ev, const uint8_t* rows40, int64_t n, int32_t local,
                                int64_t* scores) {
  if (!ctx || !ev || n < 0 || n >= ((int64_t)1 << 31) || (n > 0 && (!rows40 || !scores))) return YRWI_E_ARG;
  EVENT_LOCK(ctx);
  if (n == 0) return 0;
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  if (int rc = grow_host_table(ctx, ev, n)) return rc;
  uint8_t* d_rows = arena_alloc<uint8_t>(L, n * YRWI_ROW_BYTES);
  int64_t* d_sc = arena_alloc<int64_t>(L, n);
  EvDev* d_ev = arena_alloc<EvDev>(L, 1);
  EvJob* d_job = arena_alloc<EvJob>(L, 1);
  int32_t* d_jb = arena_alloc<int32_t>(L, 2);
  int32_t* d_status = arena_alloc<int32_t>(L, 1);
  if (!d_rows || !d_sc || !d_ev || !d_job || !d_jb || !d_status) return ctx->fail(YRWI_E_NOMEM, "arena");
  uint8_t* stg = stage_reserve(L, &L->out_stage, (size_t)n * YRWI_ROW_BYTES, true);
  if (!stg) return ctx->take(L, YRWI_E_HIP);
  std::memcpy(stg, rows40, (size_t)n * YRWI_ROW_BYTES);
  hipStream_t s = L->stream;
  HIPCHK(ctx, hipMemcpyAsync(d_rows, stg, (size_t)n * YRWI_ROW_BYTES, hipMemcpyHostToDevice, s));
  EvJob J{};
  J.ev = 0;
  J.local = local != 0;
  J.rows = d_rows;
  J.n = n;
  J.scores = d_sc;
  std::vector<EvDev> hev{ev->h};
  std::vector<EvJob> jobs{J};
  std::vector<int32_t> jb{0, 1};
  if (upload(L, d_ev, hev, d_job, jobs, d_jb, jb)) return ctx->take(L, YRWI_E_HIP);
  if (launch_event_add(d_ev, d_job, d_jb, 1, d_status, s)) return ctx->fail(YRWI_E_HIP, "event_order launch");
  int32_t st = 0;
  HIPCHK(ctx, hipMemcpyAsync(&st, d_status, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(ctx, hipMemcpyAsync(scores, d_sc, (size_t)n * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(ctx, lane_sync(L));
  ev->hosts_bound += n;
  if (st == YRWI_E_HASH) return ctx->fail(st, "container: url hash is not well-formed Base64");
  if (st == YRWI_E_NULL_LANGUAGE) return ctx->fail(st, "container: row with empty language cell (reference NPE)");
  if (st == YRWI_E_CAPACITY) return ctx->fail(st, "event tables full: max_postings too small");
  return st;
}

extern "C" int yrwi_event_authority(yrwi_ctx* ctx, yrwi_event* ev, const uint8_t* hosts6, int32_t n, int32_t* out) {
  if (!ctx || !ev || n < 0 || (n > 0 && (!hosts6 || !out))) return YRWI_E_ARG;
  EVENT_LOCK(ctx);
  if (n == 0) return 0;
  std::vector<uint64_t> keys((size_t)n);
  for (int32_t i = 0; i < n; i++) {
    uint64_t h = 0;
    for (int j = 0; j < 6; j++) {
      const int a = AHP[hosts6[6 * (size_t)i + (size_t)j]];
      if (a < 0) return ctx->fail(YRWI_E_HASH, "host hash is not well-formed Base64");
      h = (h << 6) | (uint64_t)a;
    }
    keys[(size_t)i] = h + 1;  // the host tables' key (host36 + 1)
  }
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  uint64_t* d_keys = arena_alloc<uint64_t>(L, n);
  int32_t* d_out = arena_alloc<int32_t>(L, n);
  EvDev* d_ev = arena_alloc<EvDev>(L, 1);
  if (!d_keys || !d_out || !d_ev) return ctx->fail(YRWI_E_NOMEM, "arena");
  std::vector<EvDev> hev{ev->h};
  if (upload(L, d_ev, hev, d_keys, keys)) return ctx->take(L, YRWI_E_HIP);
  if (launch_event_authority(d_ev, d_keys, n, d_out, L->stream)) return ctx->fail(YRWI_E_HIP, "authority launch");
  HIPCHK(ctx, hipMemcpyAsync(out, d_out, (size_t)n * 4, hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, lane_sync(L));
  return 0;
}

extern "C" int yrwi_event_source(yrwi_ctx* ctx, yrwi_event* ev, const uint8_t* urls12, int32_t n, int32_t* arrival,
                                 int32_t* row) {
  if (!ctx || !ev || n < 0 || (n > 0 && (!urls12 || !arrival || !row))) return YRWI_E_ARG;
  if (n == 0) return 0;
  if (!ev->h.ukey) return ctx->fail(YRWI_E_ARG, "an order-only event has no url set");
  EVENT_LOCK(ctx);
  std::vector<uint64_t> hi((size_t)n);
  std::vector<uint8_t> lo((size_t)n);
  for (int32_t i = 0; i < n; i++) {
    KeyT k;
    if (!key_of(urls12 + 12 * (size_t)i, &k)) return ctx->fail(YRWI_E_HASH, "url hash is not well-formed Base64");
    hi[(size_t)i] = k.hi;
    lo[(size_t)i] = (uint8_t)k.lo;
  }
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  uint64_t* d_hi = arena_alloc<uint64_t>(L, n);
  uint8_t* d_lo = arena_alloc<uint8_t>(L, n);
  uint64_t* d_out = arena_alloc<uint64_t>(L, n);
  EvDev* d_ev = arena_alloc<EvDev>(L, 1);
  if (!d_hi || !d_lo || !d_out || !d_ev) return ctx->fail(YRWI_E_NOMEM, "arena");
  std::vector<EvDev> hev{ev->h};
  if (upload(L, d_ev, hev, d_hi, hi, d_lo, lo)) return ctx->take(L, YRWI_E_HIP);
  if (launch_event_where(d_ev, d_hi, d_lo, n, d_out, L->stream)) return ctx->fail(YRWI_E_HIP, "event_source launch");
  std::vector<uint64_t> v((size_t)n);
  HIPCHK(ctx, hipMemcpyAsync(v.data(), d_out, (size_t)n * 8, hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, lane_sync(L));
  for (int32_t i = 0; i < n; i++) {
    const uint64_t x = v[(size_t)i];
    arrival[i] = x == ~0ull ? -1 : (int32_t)(x >> 32);
    row[i] = x == ~0ull ? -1 : (int32_t)(uint32_t)x;
  }
  return 0;
}

extern "C" int yrwi_event_result(yrwi_ctx* ctx, yrwi_event* ev, yrwi_hit* out, int32_t maxn, int32_t* nout,
                                 yrwi_event_info* info) {
  if (!ctx || !ev || maxn < 0 || (maxn > 0 && !out)) return YRWI_E_ARG;
  EVENT_LOCK(ctx);
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  EvState S;
  HIPCHK(ctx, hipMemcpyAsync(&S, ev->h.st, sizeof(S), hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, lane_sync(L));
  const int32_t n = std::min(S.nstack, maxn);
  if (n > 0) {
    HIPCHK(ctx, hipMemcpyAsync(out, ev->h.stack + (int64_t)S.cur * ev->k, sizeof(yrwi_hit) * (size_t)n,
                               hipMemcpyDeviceToHost, L->stream));
    HIPCHK(ctx, lane_sync(L));
  }
  if (nout) *nout = n;
  if (info) {
    std::memcpy(info->flagcount, S.flagcount, sizeof(info->flagcount));
    info->postings_in = S.nin;
    info->admitted_local = S.nadmit_local;
    info->admitted_remote = S.nadmit_remote;
    info->remote_arrivals = S.nremote;
    info->maxdomcount = S.maxdom;
    info->max_distance = (S.hasA && S.P > 0) ? std::abs(S.P - S.A) : 0;
    info->err = S.err;
    info->stack_size = S.nstack;
  }
  return 0;
}

namespace {

uint64_t host6(const yrwi_hit& h) {
  uint64_t v = 0;
  for (int j = 6; j < 12; j++) v = v << 8 | h.urlhash[j];
  return v;
}
// ReverseElement.compareTo (WeakPriorityBlockingQueue.java:414-425): weight, then hashCode
int rev_cmp(const yrwi_hit& a, const yrwi_hit& b) {
  if (std::memcmp(a.urlhash, b.urlhash, 12) == 0) return 0;
  if (a.score != b.score) return a.score > b.score ? -1 : 1;
  if (a.tiebreak != b.tiebreak) return a.tiebreak > b.tiebreak ? -1 : 1;
  return 0;
}
// WeakPriorityBlockingQueue.put (:119-134) into a host queue bounded by max_results_rwi
void dd_put(std::vector<DDEntry>& q, const DDEntry& e) {
  size_t lo = 0;
  while (lo < q.size() && rev_cmp(q[lo].h, e.h) < 0) lo++;
  if (lo < q.size() && rev_cmp(q[lo].h, e.h) == 0) return;  // the TreeSet holds an equal element
  for (const DDEntry& x : q)
    if (rev_cmp(x.h, e.h) == 0) return;
  q.insert(q.begin() + (std::ptrdiff_t)lo, e);
  if ((int32_t)q.size() > YRWI_MAX_K) q.pop_back();
}

}  // namespace

extern "C" int yrwi_event_pull(yrwi_ctx* ctx, yrwi_event* ev, int32_t skip_double_dom, yrwi_hit* out, int32_t maxn,
                               int32_t* nout) {
  if (!ctx || !ev || maxn < 0 || (maxn > 0 && !out) || !nout) return YRWI_E_ARG;
  EVENT_LOCK(ctx);
  *nout = 0;
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  EvState S;
  HIPCHK(ctx, hipMemcpyAsync(&S, ev->h.st, sizeof(S), hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, lane_sync(L));
  if (S.err) return ctx->fail(S.err, "event tables overflowed earlier");
  std::vector<yrwi_hit> stk((size_t)S.nstack);
  if (S.nstack > 0) {
    HIPCHK(ctx, hipMemcpyAsync(stk.data(), ev->h.stack + (int64_t)S.cur * ev->k, sizeof(yrwi_hit) * stk.size(),
                               hipMemcpyDeviceToHost, L->stream));
    HIPCHK(ctx, lane_sync(L));
  }
  // pullOneRWI(skipDoubleDom) (SearchEvent.java:1297-1394), maxn times or until null
  size_t p = 0;  // entries polled from rwiStack
  int32_t n = 0;
  while (n < maxn) {
    bool got = false;
    for (int c = 0; p < stk.size() && c < 10; c++) {  // pollloop (:1305)
      const yrwi_hit& rwi = stk[p++];
      if (!skip_double_dom) {
        out[n++] = rwi;
        got = true;
        break;
      }
      auto it = ev->dd.find(host6(rwi));
      if (it == ev->dd.end()) {  // first appearance of the host (:1320-1332)
        ev->dd.emplace(host6(rwi), std::vector<DDEntry>());
        out[n++] = rwi;
        got = true;
        break;
      }
      dd_put(it->second, DDEntry{rwi, ev->dd_next++});  // second appearance (:1335,1338)
    }
    if (got) continue;
    if (ev->dd.empty()) break;  // :1343
    // best head over the host queues (:1349-1368): largest weight; equal heads by
    // queue order, then the earliest queued (the reference walks a ConcurrentHashMap)
    auto best = ev->dd.end();
    for (auto it = ev->dd.begin(); it != ev->dd.end(); ++it) {
      if (it->second.empty()) continue;
      if (best == ev->dd.end()) { best = it; continue; }
      const DDEntry& a = it->second.front();
      const DDEntry& b = best->second.front();
      const int c = rev_cmp(a.h, b.h);
      if (c < 0 || (c == 0 && a.seq < b.seq)) best = it;
    }
    if (best == ev->dd.end()) break;
    out[n++] = best->second.front().h;  // m.poll() (:1377)
    best->second.erase(best->second.begin());
    if (best->second.empty()) ev->dd.erase(best);  // sizeAvailable() == 0 (:1378-1383)
  }
  *nout = n;
  // the polled entries leave the device stack: the rest moves to the other half
  if (p > 0) {
    const int32_t rest = S.nstack - (int32_t)p, nc = 1 - S.cur;
    if (rest > 0)
      HIPCHK(ctx, hipMemcpyAsync(ev->h.stack + (int64_t)nc * ev->k, ev->h.stack + (int64_t)S.cur * ev->k + (int64_t)p,
                                 sizeof(yrwi_hit) * (size_t)rest, hipMemcpyDeviceToDevice, L->stream));
    const int32_t v[2] = {rest, nc};
    static_assert(offsetof(EvState, cur) == offsetof(EvState, nstack) + 4, "nstack, cur adjacent");
    HIPCHK(ctx, hipMemcpyAsync(reinterpret_cast<uint8_t*>(ev->h.st) + offsetof(EvState, nstack), v, sizeof(v),
                               hipMemcpyHostToDevice, L->stream));
    HIPCHK(ctx, lane_sync(L));
  }
  return 0;
}

extern "C" void yrwi_event_close(yrwi_ctx* ctx, yrwi_event* ev) {
  if (!ev) return;
  if (ctx) {
    EVENT_LOCK(ctx);
    hipSetDevice(ctx->device);
    if (ev->pooled) {
      // the event's last call synchronised its lane (lanes[0]); its block is reused
      // by the next order-only event, zeroed on that lane's stream first
      std::lock_guard<std::mutex> lk(ctx->ev_pool_mu);
      if (ctx->ev_pool.size() < 64) {
        ctx->ev_pool.emplace_back(ev->bytes, ev->mem);
        delete ev;
        return;
      }
    }
    drain(ctx);
    lane_sync(ctx->lanes[0]);
  }
  hipFree(ev->mem);
  delete ev;
}
