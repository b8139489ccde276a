// yrwi_host.cpp -- host runtime of libyrwi: index residency, query planning
// (the Java-side decisions of TermSearch / joinContainers / joinConstructive),
// batched device execution and the C ABI declared in include/yrwi.h.
//
// Planning rules restated here (paths relative to /root/reference/source/net/yacy):
//   J1  AbstractIndex.searchConjunction :96-128, TermSearch :42-70
//       (HandleSet: term hashes are a sorted set; a missing include term empties
//        the result, a missing exclude term disables exclusion)
//   J2  ReferenceContainer.joinContainers :334-366 (TreeMap key (int)(size*1000+i))
//   J3  ReferenceContainer.joinConstructive :406-416 (int-wrapping step counts)
// Everything per posting runs on the GPU (yrwi_kernels.hip).

#include "yrwi_host.h"

using namespace yrwi;

// ===================================================================== profile
extern "C" void yrwi_profile_default(yrwi_profile* p) {
  std::memset(p, 0, sizeof(*p));
  p->coeff_appemph = 5; p->coeff_appurl = 12; p->coeff_app_dc_creator = 1;
  p->coeff_app_dc_description = 10; p->coeff_app_dc_subject = 2; p->coeff_app_dc_title = 14;
  p->coeff_authority = 5; p->coeff_cathasapp = 0; p->coeff_cathasaudio = 0; p->coeff_cathasimage = 0;
  p->coeff_cathasvideo = 0; p->coeff_catindexof = 0; p->coeff_date = 9; p->coeff_domlength = 10;
  p->coeff_hitcount = 1; p->coeff_language = 2; p->coeff_llocal = 0; p->coeff_lother = 7;
  p->coeff_phrasesintext = 0; p->coeff_posinphrase = 0; p->coeff_posintext = 4; p->coeff_posofphrase = 0;
  p->coeff_termfrequency = 8; p->coeff_urlcomps = 7; p->coeff_urllength = 6; p->coeff_worddistance = 10;
  p->coeff_wordsintext = 3; p->coeff_wordsintitle = 2; p->coeff_urlcompintoplist = 2;
  p->coeff_descrcompintoplist = 2; p->coeff_prefer = 0; p->coeff_citation = 10;
}

extern "C" void yrwi_profile_all_zero(yrwi_profile* p) { std::memset(p, 0, sizeof(*p)); }

// NumberTools.parseIntDecSubstring (NumberTools.java:91-124); false on NumberFormatException
static bool parse_int_dec(const std::string& s, size_t start, int32_t* out) {
  size_t end = s.size();
  if (end <= start) return false;
  size_t i = start;
  while (i < end && s[i] == ' ') i++;
  if (i >= end) return false;
  int64_t result = 0;
  bool neg = false;
  int64_t limit = -2147483647LL;
  char first = s[i];
  if (first < '0') {
    if (first == '-') { neg = true; limit = -2147483648LL; }
    else if (first != '+') return false;
    i++;
    if (i == end) return false;
  }
  int64_t multmin = limit / 10;
  while (i < end) {
    char c = s[i++];
    if (c < '0' || c > '9') break;
    int d = c - '0';
    if (result < multmin) return false;
    result *= 10;
    if (result < limit + d) return false;
    result -= d;
  }
  *out = (int32_t)(neg ? result : -result);
  return true;
}

// RankingProfile(String prefix, String profile) (RankingProfile.java:127-189)
extern "C" int yrwi_profile_parse(const char* prefix, const char* ext, yrwi_profile* out) {
  yrwi_profile_default(out);
  if (!ext || !*ext) return 0;
  std::string profile(ext);
  if (profile[0] == '{' && profile.back() == '}') profile = profile.substr(1, profile.size() - 2);
  auto trim = [](const std::string& x) {
    size_t a = 0, b = x.size();
    while (a < b && (unsigned char)x[a] <= ' ') a++;
    while (b > a && (unsigned char)x[b - 1] <= ' ') b--;
    return x.substr(a, b - a);
  };
  profile = trim(profile);
  std::vector<std::string> elts;
  char sep = (profile.find('&') != std::string::npos && profile.find('&') > 0) ? '&' : ',';
  {
    // String.split drops trailing empty strings; empty elements are harmless here
    size_t st = 0;
    while (true) {
      size_t p = profile.find(sep, st);
      elts.push_back(profile.substr(st, p == std::string::npos ? std::string::npos : p - st));
      if (p == std::string::npos) break;
      st = p + 1;
    }
  }
  std::string pre = prefix ? prefix : "";
  std::map<std::string, int32_t> coeff;
  for (auto& elt : elts) {
    std::string e = trim(elt);
    if (pre.empty() || e.compare(0, pre.size(), pre) == 0) {
      size_t p = e.find('=');
      if (p != std::string::npos && p > 0 && e.size() > p + 1) {
        int32_t v;
        if (parse_int_dec(e, p + 1, &v)) coeff[e.substr(pre.size(), p - pre.size())] = v;
      }
    }
  }
  struct F { const char* n; int32_t yrwi_profile::*f; };
  static const F fields[] = {
      {"domlength", &yrwi_profile::coeff_domlength}, {"date", &yrwi_profile::coeff_date},
      {"wordsintitle", &yrwi_profile::coeff_wordsintitle}, {"wordsintext", &yrwi_profile::coeff_wordsintext},
      {"phrasesintext", &yrwi_profile::coeff_phrasesintext}, {"llocal", &yrwi_profile::coeff_llocal},
      {"lother", &yrwi_profile::coeff_lother}, {"urllength", &yrwi_profile::coeff_urllength},
      {"urlcomps", &yrwi_profile::coeff_urlcomps}, {"hitcount", &yrwi_profile::coeff_hitcount},
      {"posintext", &yrwi_profile::coeff_posintext}, {"posofphrase", &yrwi_profile::coeff_posofphrase},
      {"posinphrase", &yrwi_profile::coeff_posinphrase}, {"authority", &yrwi_profile::coeff_authority},
      {"worddistance", &yrwi_profile::coeff_worddistance}, {"appurl", &yrwi_profile::coeff_appurl},
      {"appdescr", &yrwi_profile::coeff_app_dc_title}, {"appauthor", &yrwi_profile::coeff_app_dc_creator},
      {"apptags", &yrwi_profile::coeff_app_dc_subject}, {"appref", &yrwi_profile::coeff_app_dc_description},
      {"appemph", &yrwi_profile::coeff_appemph}, {"catindexof", &yrwi_profile::coeff_catindexof},
      {"cathasimage", &yrwi_profile::coeff_cathasimage}, {"cathasaudio", &yrwi_profile::coeff_cathasaudio},
      {"cathasvideo", &yrwi_profile::coeff_cathasvideo}, {"cathasapp", &yrwi_profile::coeff_cathasapp},
      {"tf", &yrwi_profile::coeff_termfrequency}, {"urlcompintoplist", &yrwi_profile::coeff_urlcompintoplist},
      {"descrcompintoplist", &yrwi_profile::coeff_descrcompintoplist}, {"prefer", &yrwi_profile::coeff_prefer},
      {"language", &yrwi_profile::coeff_language}, {"citation", &yrwi_profile::coeff_citation}};
  for (auto& f : fields) {
    auto it = coeff.find(f.n);
    if (it != coeff.end()) out->*(f.f) = it->second;
  }
  return 0;
}

// ===================================================================== context
extern "C" int yrwi_get_unique_id(uint8_t id[128]) {
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return YRWI_E_RCCL;
  static_assert(sizeof(u) == 128, "ncclUniqueId size");
  std::memcpy(id, &u, 128);
  return 0;
}

static void close_lanes(yrwi_ctx* ctx) {
  for (Lane* L : ctx->lanes) L->wait();
  for (Lane* L : ctx->lanes) {
    L->stop();
    if (L->stream) hipStreamSynchronize(L->stream);
    if (L->comm && L->comm != ctx->lanes[0]->comm) ncclCommDestroy(L->comm);
  }
  if (!ctx->lanes.empty() && ctx->lanes[0]->comm) ncclCommDestroy(ctx->lanes[0]->comm);
  for (Lane* L : ctx->lanes) {
    if (L->loop) loop_leave(L->loop);
    for (auto e : L->coll_ev)
      if (e) hipEventDestroy(e);
    L->arena.release();
    for (auto e : L->evpool) hipEventDestroy(e);
    if (L->stage.p) hipHostFree(L->stage.p);
    if (L->out_stage.p) hipHostFree(L->out_stage.p);
    if (L->down_stage.p) hipHostFree(L->down_stage.p);
    if (L->sync_ev) hipEventDestroy(L->sync_ev);
    if (L->stream && L->own_stream) hipStreamDestroy(L->stream);
    delete L;
  }
  ctx->lanes.clear();
}

// What a lane's first batch would otherwise set up inside the caller's first
// timed batches: its wait event, the pinned staging buffers (uploads, joined-size
// readbacks, result landing), the first scratch chunk and the stream's hardware
// queue (a first operation on it).  Runs on the lane's own thread at open.
static int warm_lane(Lane* L) {
  if (hipSetDevice(L->device) != hipSuccess) return L->fail(YRWI_E_HIP, "hipSetDevice");
  constexpr size_t kStage = (size_t)4 << 20;
  if (!stage_reserve(L, &L->stage, kStage, false) || !stage_reserve(L, &L->down_stage, kStage, false) ||
      !stage_reserve(L, &L->out_stage, kStage, false))
    return YRWI_E_HIP;
  uint8_t* p = L->arena.alloc(256);
  if (!p) return L->fail(YRWI_E_NOMEM, "scratch");
  HIPCHK(L, hipMemsetAsync(p, 0, 256, L->stream));
  HIPCHK(L, lane_sync(L));
  L->arena.reset();
  return 0;
}

// why the calling thread's last yrwi_open / yrwi_open_shard failed (no context to
// hold it): yrwi_last_error(NULL)
static thread_local std::string t_open_error;
static void set_open_error(const std::string& m) { t_open_error = m; }

static int open_common(int device, int rank, int world, yrwi_ctx** out) {
  *out = nullptr;
  t_open_error.clear();
  if (hipSetDevice(device) != hipSuccess) {
    set_open_error("hipSetDevice(" + std::to_string(device) + ") failed");
    return YRWI_E_HIP;
  }
  yrwi_ctx* ctx = new yrwi_ctx();
  ctx->device = device;
  ctx->rank = rank;
  ctx->world = world;
  // Eight lanes, sharded or not (C2, 400-step runs on one box: 0.76-0.80 ms per
  // batch with eight in flight, 0.80-0.86 with four, 1.0-1.25 with two: a lane's
  // host planning and its mid-batch wait for the joined sizes leave the device
  // idle unless enough other batches queue work).  The collectives of the lanes'
  // batch parts are enqueued in one total order on every rank (CollTurn,
  // yrwi_host.h).  Scratch: 128 GiB over all lanes (scratch_budget).
  const char* e = getenv("YRWI_LANES");
  const int nl = e ? std::max(1, std::min(16, atoi(e))) : 8;
  for (int l = 0; l < nl; l++) {
    Lane* L = new Lane();
    L->device = device;
    L->rank = rank;
    L->world = world;
    ctx->lanes.push_back(L);
    if (hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking) != hipSuccess) {
      close_lanes(ctx);
      delete ctx;
      set_open_error("hipStreamCreateWithFlags failed");
      return YRWI_E_HIP;
    }
    L->hostreg = &ctx->hostreg;
    L->turn = &ctx->turn;
    L->scratch_hint = &ctx->scratch_hint;
    L->scratch_total = &ctx->scratch_total;
    L->nlanes = nl;
    L->start_worker();
  }
  for (Lane* L : ctx->lanes) L->submit([L] { L->rc = warm_lane(L); });
  int wrc = 0;
  for (Lane* L : ctx->lanes) {
    L->wait();
    if (L->rc && !wrc) {
      wrc = L->rc;
      set_open_error("lane set-up: " + L->err);
    }
  }
  if (wrc) {
    close_lanes(ctx);
    delete ctx;
    return wrc;
  }
  ctx->stream = ctx->lanes[0]->stream;
  *out = ctx;
  return 0;
}

extern "C" int yrwi_open(int device, yrwi_ctx** out) { return open_common(device, 0, 1, out); }

extern "C" int yrwi_open_shard(int device, int rank, int world, const uint8_t nccl_id[128], yrwi_ctx** out) {
  if (world < 1 || (world & (world - 1)) || world > 64 || rank < 0 || rank >= world) return YRWI_E_ARG;
  int rc = open_common(device, rank, world, out);
  if (rc) return rc;
  yrwi_ctx* ctx = *out;
  const bool loop = world > 1 && std::memcmp(nccl_id, LOOP_TAG, sizeof(LOOP_TAG)) == 0;
  // YRWI_COLL_SELF=1: a world-1 context runs the sharded protocol over a real
  // 1-rank communicator (tests: RCCL on a one-GPU box; Lane::sharded)
  const char* cs = getenv("YRWI_COLL_SELF");
  ctx->sharded = world > 1 || (cs && atoi(cs));
  for (Lane* L : ctx->lanes) L->sharded = ctx->sharded;
  if (world > 1) {  // list-size exchanges through host shared memory (the ranks of one node)
    ctx->hostx = hostx_open(nccl_id, world, rank);
    for (Lane* L : ctx->lanes) L->hostx = ctx->hostx;
  }
  if (loop) {
    // in-process loopback group (tests: several shards on one GPU), one per lane
    bool ok = true;
    for (size_t l = 0; ok && l < ctx->lanes.size(); l++) {
      uint8_t id[128];
      std::memcpy(id, nccl_id, 128);
      id[127] ^= (uint8_t)l;
      ctx->lanes[l]->loop = loop_join(id, world, rank);
      ok = ctx->lanes[l]->loop != nullptr;
    }
    ctx->transport = YRWI_TRANSPORT_LOOPBACK;
    if (!ok) {
      yrwi_close(ctx);
      *out = nullptr;
      return YRWI_E_ARG;
    }
  } else if (ctx->sharded) {
    ctx->transport = YRWI_TRANSPORT_RCCL;
    // The transport is decided from facts every rank sees alike, before any
    // collective: ranks on ONE device (RCCL refuses a duplicate GPU) or an id
    // tagged YRWI-HOSTSTAGE exchange through host shared memory; ranks on
    // distinct devices use RCCL, and an RCCL failure there is an error, never a
    // silent switch to the host path.
    const bool staged = world > 1 && std::memcmp(nccl_id, STAGE_TAG, sizeof(STAGE_TAG)) == 0;
    int peers = -1;
    if (world > 1 && ctx->hostx) {
      char bus[32] = {0};
      int64_t devid = 0;
      if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus), device) == hipSuccess) {
        uint64_t h = 1469598103934665603ull;  // FNV-1a of "dddd:bb:dd.f"
        for (const char* c = bus; *c; c++) h = (h ^ (uint8_t)*c) * 1099511628211ull;
        devid = (int64_t)(h >> 1) | 1;
      } else {
        devid = -(int64_t)rank - 1;  // unknown: distinct from every other rank's
      }
      peers = hostx_device_peers(ctx->hostx, devid, 120.0);
    }
    ctx->device_peers = peers;
    if (staged || peers > 0) {
      const char* why = staged ? "host-staged group id" : "ranks share a device";
      ctx->devx = (ctx->hostx && (staged ? hostx_wait_attached(ctx->hostx, 120.0) : true))
                      ? devx_open(nccl_id, world, rank, ctx->hostx) : nullptr;
      if (!ctx->devx) {
        set_open_error(std::string("host-staged collectives (") + why + ") unavailable: " +
                       (ctx->hostx ? "shared-memory segment" : "no host mailbox"));
        yrwi_close(ctx);
        *out = nullptr;
        return YRWI_E_RCCL;
      }
      for (Lane* L : ctx->lanes) L->devx = ctx->devx;
      ctx->transport = YRWI_TRANSPORT_HOSTSTAGED;
      if (!staged) fprintf(stderr, "yrwi: rank %d of %d: %s -- collectives host-staged through /dev/shm\n", rank,
                           world, why);
      return 0;
    }
    ncclUniqueId u;
    std::memcpy(&u, nccl_id, 128);
    ncclComm_t c0 = nullptr;
    const ncclResult_t irc = ncclCommInitRank(&c0, world, u, rank);
    if (irc != ncclSuccess) {
      set_open_error(std::string("ncclCommInitRank (rank ") + std::to_string(rank) + " of " + std::to_string(world) +
                     "): " + ncclGetErrorString(irc));
      yrwi_close(ctx);
      *out = nullptr;
      return YRWI_E_RCCL;
    }
    bool ok = true;
    ctx->lanes[0]->comm = c0;
    // the mailbox only works if every rank mapped the same segment (one node, one
    // /dev/shm): every rank opened it before the init above, so after it each
    // rank sees world attachments or not; all ranks agree (min over the ranks)
    // and drop the mailbox together if any one saw fewer (device all-gather then)
    if (world > 1) {
      int32_t* d_flag = nullptr;
      int32_t flag = hostx_attached(ctx->hostx) == world ? 1 : 0;
      ok = hipMalloc(&d_flag, 4) == hipSuccess;
      ok = ok && hipMemcpy(d_flag, &flag, 4, hipMemcpyHostToDevice) == hipSuccess;
      ok = ok && ncclAllReduce(d_flag, d_flag, 1, ncclInt32, ncclMin, c0, ctx->stream) == ncclSuccess;
      ok = ok && hipMemcpyAsync(&flag, d_flag, 4, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess;
      ok = ok && hipStreamSynchronize(ctx->stream) == hipSuccess;
      if (d_flag) hipFree(d_flag);
      if (ok && !flag && ctx->hostx) {
        hostx_close(ctx->hostx, rank == 0);  // some rank never mapped it: nobody else unlinks the name
        ctx->hostx = nullptr;
        for (Lane* L : ctx->lanes) L->hostx = nullptr;
      }
    }
    // one communicator per lane: lanes issue their collectives independently.  If
    // the split fails (the same way on every rank), the lanes share c0 -- still
    // safe: the collective turn lets one batch part at a time enqueue, in one
    // total order on every rank (close_lanes destroys c0 once).
    bool split = ok;
    for (size_t l = 1; split && l < ctx->lanes.size(); l++)
      split = ncclCommSplit(c0, 0, rank, &ctx->lanes[l]->comm, nullptr) == ncclSuccess;
    if (ok && !split)
      for (size_t l = 1; l < ctx->lanes.size(); l++) {
        if (ctx->lanes[l]->comm && ctx->lanes[l]->comm != c0) ncclCommDestroy(ctx->lanes[l]->comm);
        ctx->lanes[l]->comm = c0;
      }
    if (!ok) {
      set_open_error("RCCL group set-up after ncclCommInitRank failed (mailbox agreement all-reduce)");
      yrwi_close(ctx);
      *out = nullptr;
      return YRWI_E_RCCL;
    }
  }
  return 0;
}

extern "C" int yrwi_shard_info(yrwi_ctx* ctx, yrwi_transport_info* out) {
  if (!ctx || !out) return YRWI_E_ARG;
  std::memset(out, 0, sizeof(*out));
  out->transport = ctx->transport;
  out->rank = ctx->rank;
  out->world = ctx->world;
  out->lanes = (int32_t)ctx->lanes.size();
  out->device_peers = ctx->device_peers;
  out->mailbox = ctx->hostx ? 1 : 0;
  ncclComm_t c0 = ctx->lanes.empty() ? nullptr : ctx->lanes[0]->comm;
  if (c0) {
    int n = 0;
    if (ncclCommCount(c0, &n) == ncclSuccess) out->rccl_ranks = n;
    for (size_t l = 0; l < ctx->lanes.size(); l++)
      out->lanes_own_comm += ctx->lanes[l]->comm && (l == 0 || ctx->lanes[l]->comm != c0);
  }
  hipDeviceGetPCIBusId(out->pci_bus_id, (int)sizeof(out->pci_bus_id), ctx->device);
  return 0;
}

extern "C" void yrwi_close(yrwi_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  close_lanes(ctx);
  // unlinked once every rank mapped it (hostx_open); rank 0 unlinks it again in
  // case some rank never did (ENOENT is harmless)
  hostx_close(ctx->hostx, ctx->rank == 0);
  ctx->hostx = nullptr;
  devx_close(ctx->devx, ctx->rank == 0);
  ctx->devx = nullptr;
  for (auto& b : ctx->ev_pool) hipFree(b.second);
  ctx->ev_pool.clear();
  if (ctx->host_key) hipFree(ctx->host_key);
  ctx->index_mem.release();
  if (ctx->uid_all) hipFree(ctx->uid_all);
  if (ctx->head_all) hipFree(ctx->head_all);
  if (ctx->bm_all) hipFree(ctx->bm_all);
  if (ctx->dkhi) hipFree(ctx->dkhi);
  if (ctx->dklo) hipFree(ctx->dklo);
  delete ctx;
}

extern "C" const char* yrwi_last_error(yrwi_ctx* ctx) {
  if (ctx) return ctx->err.c_str();
  return t_open_error.empty() ? "null context" : t_open_error.c_str();
}

// ======================================================================= index
extern "C" int yrwi_put_list(yrwi_ctx* ctx, const uint8_t term[12], const uint8_t* rows40, int64_t n, int sorted) {
  if (!ctx || !term || n < 0 || (n > 0 && !rows40)) return YRWI_E_ARG;
  KeyT tk;
  if (!key_of(term, &tk)) return ctx->fail(YRWI_E_HASH, "term hash is not well-formed Base64");
  if (n > MAX_LIST) return ctx->fail(YRWI_E_LIMIT, "list longer than 53,687,091 rows (RowSet.importRowSet)");
  hipSetDevice(ctx->device);
  drain(ctx);  // in-flight batches read the list table
  if (n == 0) {
    auto it = ctx->lists.find(tk);
    if (it != ctx->lists.end()) {
      index_changed(ctx, tk, it->second.n, false);
      ctx->npostings -= it->second.n;
      ctx->lists.erase(it);
    }
    return 0;
  }
  std::vector<uint8_t> tmp;
  const uint8_t* src = rows40;
  if (!sorted) {
    // RowSet sort; on duplicate url hashes the first occurrence wins (RowSet.mergeEnum)
    std::vector<std::pair<KeyT, int64_t>> ks((size_t)n);
    for (int64_t i = 0; i < n; i++) {
      if (!key_of(rows40 + i * 40, &ks[(size_t)i].first)) return ctx->fail(YRWI_E_HASH, "malformed url hash");
      ks[(size_t)i].second = i;
    }
    std::stable_sort(ks.begin(), ks.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    tmp.reserve((size_t)n * 40);
    for (size_t i = 0; i < ks.size(); i++) {
      if (i > 0 && ks[i].first == ks[i - 1].first) continue;
      tmp.insert(tmp.end(), rows40 + ks[i].second * 40, rows40 + ks[i].second * 40 + 40);
    }
    src = tmp.data();
    n = (int64_t)(tmp.size() / 40);
  }
  ListRec L;
  L.n = n;
  L.rows = ctx->index_mem.alloc((size_t)n * 40);
  L.khi = reinterpret_cast<uint64_t*>(ctx->index_mem.alloc((size_t)n * 8));
  L.klo = ctx->index_mem.alloc((size_t)n);
  int32_t* derr = reinterpret_cast<int32_t*>(ctx->index_mem.alloc(4));
  if (!L.rows || !L.khi || !L.klo || !derr) return ctx->fail(YRWI_E_NOMEM, "device index allocation failed");
  HIPCHK(ctx, hipMemcpyAsync(L.rows, src, (size_t)n * 40, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync(derr, 0, 4, ctx->stream));
  if (launch_validate_rows(L.rows, n, L.khi, L.klo, derr, ctx->stream)) return ctx->fail(YRWI_E_HIP, "validate launch");
  int32_t herr = 0;
  HIPCHK(ctx, hipMemcpyAsync(&herr, derr, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  if (herr & 1) return ctx->fail(YRWI_E_HASH, "url hash is not well-formed Base64");
  if (herr & 2) return ctx->fail(YRWI_E_NULL_LANGUAGE, "row with empty language cell (reference NPE)");
  if (herr & 4) return ctx->fail(YRWI_E_UNSORTED, "rows are not strictly ascending by url hash");
  auto it = ctx->lists.find(tk);
  const int64_t old_n = it != ctx->lists.end() ? it->second.n : 0;
  ctx->npostings -= old_n;
  ctx->lists[tk] = L;
  ctx->npostings += n;
  index_changed(ctx, tk, old_n, true);
  return 0;
}

extern "C" int yrwi_check_url_ids(yrwi_ctx* ctx, int64_t* bad, int64_t* nurls) {
  if (!ctx || !bad) return YRWI_E_ARG;
  hipSetDevice(ctx->device);
  drain(ctx);
  const int rc = check_url_ids(ctx, bad);
  if (nurls) *nurls = ctx->nurls;
  return rc;
}

extern "C" int yrwi_build_url_ids(yrwi_ctx* ctx) {
  if (!ctx) return YRWI_E_ARG;
  hipSetDevice(ctx->device);
  drain(ctx);
  return ensure_url_ids(ctx);
}

extern "C" int yrwi_list_size(yrwi_ctx* ctx, const uint8_t term[12], int64_t* n) {
  KeyT tk;
  if (!ctx || !n) return YRWI_E_ARG;
  if (!key_of(term, &tk)) return ctx->fail(YRWI_E_HASH, "term hash is not well-formed Base64");
  auto it = ctx->lists.find(tk);
  *n = it == ctx->lists.end() ? 0 : it->second.n;
  return 0;
}

extern "C" int yrwi_get_list(yrwi_ctx* ctx, const uint8_t term[12], uint8_t* rows40, int64_t cap, int64_t* n) {
  KeyT tk;
  if (!ctx || !n || cap < 0 || (cap > 0 && !rows40)) return YRWI_E_ARG;
  if (!key_of(term, &tk)) return ctx->fail(YRWI_E_HASH, "term hash is not well-formed Base64");
  // like put_list: no batch in flight (the copy below runs on lane 0's stream)
  drain(ctx);
  auto it = ctx->lists.find(tk);
  *n = it == ctx->lists.end() ? 0 : it->second.n;
  if (*n == 0) return 0;
  if (cap < *n) return ctx->fail(YRWI_E_ARG, "row buffer smaller than the list");
  hipSetDevice(ctx->device);
  HIPCHK(ctx, hipMemcpyAsync(rows40, it->second.rows, (size_t)*n * 40, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

extern "C" int64_t yrwi_realloc_events(void) { return g_realloc.load(); }

extern "C" int yrwi_index_info_get(yrwi_ctx* ctx, yrwi_index_info* info) {
  if (!ctx || !info) return YRWI_E_ARG;
  std::memset(info, 0, sizeof(*info));
  info->full_rebuilds = ctx->dict_full_builds;
  info->incremental_updates = ctx->dict_incremental;
  info->repacks = ctx->index_repacks;
  info->index_bytes = (int64_t)ctx->index_mem.capacity();
  info->index_bytes_used = (int64_t)ctx->index_mem.total_used;
  for (auto& kv : ctx->lists) info->bitmap_lists += kv.second.bm != nullptr;
  return 0;
}

extern "C" int yrwi_index_stats(yrwi_ctx* ctx, int64_t* nterms, int64_t* npostings, int64_t* device_bytes) {
  if (!ctx) return YRWI_E_ARG;
  if (nterms) *nterms = (int64_t)ctx->lists.size();
  if (npostings) *npostings = ctx->npostings;
  if (device_bytes) {
    // index memory, url ids, line heads, bitmaps, url dictionary, lane scratch
    size_t b = ctx->index_mem.capacity() + ctx->uid_cap * 4 + ctx->head_cap * 4 + ctx->bm_cap * 8 +
               ctx->dict_cap * 9;
    for (Lane* L : ctx->lanes) b += L->arena.capacity();
    *device_bytes = (int64_t)b;
  }
  return 0;
}

// ================================================================== planning
// yrwi_filter -> FilterQ (device pointers left null), the sorted unique host keys
// of siteexcludes and the sorted unique url keys of the doublecheck seed set.
void yrwi::build_filterq(const yrwi_filter& F, FilterQ* Gp, std::vector<uint64_t>* siteex, std::vector<KeyT>* urls) {
  FilterQ& G = *Gp;
  std::memset(&G, 0, sizeof(G));
  std::memcpy(G.constraint, F.constraint, 4);
  G.has_constraint = F.has_constraint != 0;
  G.all_of = F.all_of_constraint != 0;
  G.contentdom = F.contentdom;
  G.strict = F.strict_contentdom != 0;
  const size_t ll = strnlen(F.language, sizeof(F.language));
  G.lang_len = (int32_t)ll;
  std::memcpy(G.lang, F.language, ll);
  auto host_key = [](const uint8_t* h, uint64_t* k) {
    uint64_t x = 0;
    for (int j = 0; j < 6; j++) {
      if (AHP[h[j]] < 0) return false;
      x = (x << 6) | (uint64_t)AHP[h[j]];
    }
    *k = x;
    return true;
  };
  // a host hash outside the alphabet matches no row (rows are validated)
  G.has_site = F.has_sitehash != 0;
  G.has_alt = F.has_alt_sitehash != 0 && host_key(F.alt_sitehash, &G.altsite);
  if (G.has_site && !host_key(F.sitehash, &G.site)) G.site = ~0ull;
  std::vector<uint64_t>& v = *siteex;
  v.clear();
  for (int i = 0; i < F.nsiteexcludes; i++) {
    uint64_t k;
    if (host_key(F.siteexcludes + 6 * i, &k)) v.push_back(k);
  }
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  G.nsiteex = (int64_t)v.size();
  std::vector<KeyT>& u = *urls;
  u.clear();
  for (int i = 0; i < F.nurlhashes; i++) {
    KeyT k;
    if (key_of(F.urlhashes + 12 * i, &k)) u.push_back(k);
  }
  std::sort(u.begin(), u.end());
  u.erase(std::unique(u.begin(), u.end()), u.end());
  G.nurl = (int64_t)u.size();
}

static int plan_query(const yrwi_ctx* ix, Lane* ctx, const yrwi_query_desc& d, Plan* P) {
  P->maxd = d.max_distance;
  P->k = std::min<int32_t>(std::max<int32_t>(d.k, 0), YRWI_MAX_K);
  if (d.profile) P->prof = *d.profile; else yrwi_profile_default(&P->prof);
  size_t ll = strnlen(d.language, sizeof(d.language));
  P->lang_ok = ll == 2;
  P->lang[0] = ll > 0 ? (uint8_t)d.language[0] : 0;
  P->lang[1] = ll > 1 ? (uint8_t)d.language[1] : 0;
  if (d.now_ms != 0) {
    P->now_ms = d.now_ms;
  } else {
    P->now_ms = (int64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
                    std::chrono::system_clock::now().time_since_epoch()).count();
  }
  if (d.nincl < 0 || d.nexcl < 0 || d.nincl > YRWI_MAX_TERMS || d.nexcl > YRWI_MAX_TERMS)
    return ctx->fail(YRWI_E_ARG, "too many terms");
  P->filter = d.filter;
  if (const yrwi_filter* F = d.filter) {
    if (F->nsiteexcludes < 0 || F->nurlhashes < 0 || (F->nsiteexcludes > 0 && !F->siteexcludes) ||
        (F->nurlhashes > 0 && !F->urlhashes))
      return ctx->fail(YRWI_E_ARG, "filter: bad siteexcludes / urlhashes");
  }
  // HandleSet: sorted (Base64Order) set of term hashes
  int ninc = 0, nexc = 0;
  for (int i = 0; i < d.nincl; i++)
    if (!key_of(d.incl + 12 * i, &P->inc[ninc++])) return ctx->fail(YRWI_E_HASH, "include term hash not well-formed");
  for (int i = 0; i < d.nexcl; i++)
    if (!key_of(d.excl + 12 * i, &P->exc[nexc++])) return ctx->fail(YRWI_E_HASH, "exclude term hash not well-formed");
  P->has_sel = d.urlselection != nullptr && d.nurlselection > 0;
  P->sel.clear();
  P->sel_uid.clear();
  if (d.nurlselection < 0 || (d.nurlselection > 0 && !d.urlselection))
    return ctx->fail(YRWI_E_ARG, "bad urlselection");
  if (P->has_sel) {  // HandleSet urlselection: a sorted set of url hashes
    P->sel.resize((size_t)d.nurlselection);
    for (int32_t i = 0; i < d.nurlselection; i++)
      if (!key_of(d.urlselection + 12 * (size_t)i, &P->sel[(size_t)i]))
        return ctx->fail(YRWI_E_HASH, "urlselection hash not well-formed");
    std::sort(P->sel.begin(), P->sel.end());
    P->sel.erase(std::unique(P->sel.begin(), P->sel.end()), P->sel.end());
  }
  std::sort(P->inc, P->inc + ninc);
  ninc = (int)(std::unique(P->inc, P->inc + ninc) - P->inc);
  std::sort(P->exc, P->exc + nexc);
  nexc = (int)(std::unique(P->exc, P->exc + nexc) - P->exc);
  P->ninc = ninc;
  P->nexc = nexc;
  auto local = [&](const KeyT& k) -> const ListRec* {
    auto it = ix->lists.find(k);
    return (it == ix->lists.end() || it->second.n == 0) ? nullptr : &it->second;
  };
  for (int i = 0; i < ninc; i++) P->linc[i] = local(P->inc[i]);
  for (int i = 0; i < nexc; i++) P->lexc[i] = local(P->exc[i]);
  P->empty = true;
  P->postings_in = 0;
  for (int i = 0; i < ninc; i++) P->postings_in += P->linc[i] ? P->linc[i]->n : 0;
  for (int i = 0; i < nexc; i++) P->postings_in += P->lexc[i] ? P->lexc[i]->n : 0;
  return 0;
}

// A list of a query term that this url-hash shard does not hold.
static const ListRec kAbsentList{};

// The size-dependent decisions of TermSearch / joinContainers, taken on the
// GLOBAL list sizes ng_inc / ng_exc (one context: its own sizes; url-hash
// shards: the sum over all shards, so every shard takes the decisions the single
// container would -- AbstractIndex.java:108-127, ReferenceContainer.java:334-366):
//   J1  any include term without postings empties the result; any exclude term
//       without postings disables the exclusion;
//   J2  fold order by (int)(size*1000 + count), a later put overwriting an
//       equal key.
// The lists joined are the shard's own (absent ones are empty).
static void plan_finish(Plan* P, const int64_t* ng_inc, const int64_t* ng_exc) {
  P->empty = true;
  P->seq.clear();
  P->seq_ng.clear();
  P->excl.clear();
  if (P->ninc == 0) return;
  for (int i = 0; i < P->ninc; i++)
    if (ng_inc[i] == 0) return;  // conjunction: any missing term -> empty
  bool use_excl = P->nexc > 0;
  for (int i = 0; i < P->nexc; i++)
    if (ng_exc[i] == 0) use_excl = false;
  P->nexcl_g = use_excl ? P->nexc : 0;
  if (use_excl)
    for (int i = 0; i < P->nexc; i++)
      if (P->lexc[i]) P->excl.push_back(P->lexc[i]);
  // joinContainers: TreeMap<Long>((int)(size*1000 + count)); put overwrites equal keys
  std::pair<int32_t, int> tm[YRWI_MAX_TERMS];
  for (int c = 0; c < P->ninc; c++) tm[c] = {add32(mul32((int32_t)ng_inc[c], 1000), c), c};
  std::stable_sort(tm, tm + P->ninc, [](const std::pair<int32_t, int>& a, const std::pair<int32_t, int>& b) {
    return a.first < b.first;
  });
  for (int i = 0; i < P->ninc; i++) {
    if (i + 1 < P->ninc && tm[i + 1].first == tm[i].first) continue;  // the later put wins
    const int c = tm[i].second;
    P->seq_term[P->seq.size()] = c;
    P->seq.push_back(P->linc[c] ? P->linc[c] : &kAbsentList);
    P->seq_ng.push_back(ng_inc[c]);
  }
  P->empty = false;
}

// Element-wise sum of v over the url-hash shards (every rank passes vectors of
// the same length, in the same sequence of calls); identity on one context.
static int allsum_host(Lane* L, std::vector<int64_t>& v) {
  if (!L->sharded || v.empty()) return 0;
  const int hx = hostx_allsum(L, v);  // the node's shared-memory mailbox (no device collective, no turn)
  if (hx <= 0) return hx;
  const size_t n = v.size();
  int64_t* d_v = arena_alloc<int64_t>(L, (int64_t)n);
  int64_t* d_all = arena_alloc<int64_t>(L, (int64_t)n * L->world);
  if (!d_v || !d_all) return L->fail(YRWI_E_NOMEM, "arena");
  if (upload(L, d_v, v)) return YRWI_E_HIP;
  if (int rc = coll_allgather(L, d_v, d_all, n * sizeof(int64_t))) return rc;
  const uint8_t* hb = readback(L, &L->down_stage, d_all, (int64_t)n * L->world, 8, 8);
  if (!hb) return YRWI_E_HIP;
  HIPCHK(L, lane_sync(L));
  std::vector<int64_t> all(n * (size_t)L->world);
  std::memcpy(all.data(), hb, all.size() * sizeof(int64_t));
  for (size_t i = 0; i < n; i++) {
    int64_t s = 0;
    for (int r = 0; r < L->world; r++) s += all[(size_t)r * n + i];
    v[i] = s;
  }
  return 0;
}

static ChainList chain_list(const ListRec* L) { return ChainList{L->uid, L->head, L->bm, L->n}; }

// TermSearch's urlselection (yrwi_query_desc.urlselection): every selection
// query's url ids on this shard (from the url dictionary; urls it does not hold
// can match nothing) and the local sizes of its include and exclude lists
// restricted to them -- the sizes ReferenceContainerCache.get(key, urlselection)
// gives (ReferenceContainerCache.java:448-470), on which J1 / J2 / J3 decide.
static int resolve_selections(Lane* L, std::vector<Plan>& plans) {
  std::vector<size_t> qs;
  for (size_t q = 0; q < plans.size(); q++)
    if (plans[q].has_sel) qs.push_back(q);
  if (qs.empty()) return 0;
  if (begin_pass(L)) return YRWI_E_HIP;
  std::vector<uint64_t> hi;
  std::vector<uint8_t> lo;
  std::vector<size_t> off{0};
  for (size_t q : qs) {
    for (const KeyT& k : plans[q].sel) {
      hi.push_back(k.hi);
      lo.push_back((uint8_t)k.lo);
    }
    off.push_back(hi.size());
  }
  const int64_t n = (int64_t)hi.size();
  uint64_t* d_hi = arena_alloc<uint64_t>(L, n);
  uint8_t* d_lo = arena_alloc<uint8_t>(L, n);
  uint32_t* d_uid = arena_alloc<uint32_t>(L, n);
  if (!d_hi || !d_lo || !d_uid) return L->fail(YRWI_E_NOMEM, "arena");
  if (upload(L, d_hi, hi, d_lo, lo)) return YRWI_E_HIP;
  if (launch_sel_lookup(d_hi, d_lo, n, L->dkhi, L->dklo, L->dkhi ? L->nurls : 0, d_uid, L->stream))
    return L->fail(YRWI_E_HIP, "selection lookup launch");
  const uint8_t* hb = readback(L, &L->down_stage, d_uid, n, 4, 4);
  if (!hb) return YRWI_E_HIP;
  HIPCHK(L, lane_sync(L));
  std::vector<uint32_t> uids((size_t)n);
  std::memcpy(uids.data(), hb, (size_t)n * 4);
  std::vector<uint32_t> all;  // every query's ids, concatenated (ascending per query: ids keep key order)
  std::vector<int64_t> aoff;
  for (size_t i = 0; i < qs.size(); i++) {
    Plan& P = plans[qs[i]];
    P.sel_uid.clear();
    for (size_t j = off[i]; j < off[i + 1]; j++)
      if (uids[j] != 0xFFFFFFFFu) P.sel_uid.push_back(uids[j]);
    aoff.push_back((int64_t)all.size());
    all.insert(all.end(), P.sel_uid.begin(), P.sel_uid.end());
  }
  uint32_t* d_all = arena_alloc<uint32_t>(L, (int64_t)all.size());
  if (!d_all) return L->fail(YRWI_E_NOMEM, "arena");
  std::vector<SelCount> jobs;
  std::vector<std::pair<size_t, int>> who;  // (plan, list: include i or YRWI_MAX_TERMS + exclude i)
  int64_t* d_cnt = arena_alloc<int64_t>(L, (int64_t)qs.size() * 2 * YRWI_MAX_TERMS);
  if (!d_cnt) return L->fail(YRWI_E_NOMEM, "arena");
  for (size_t i = 0; i < qs.size(); i++) {
    Plan& P = plans[qs[i]];
    for (int t = 0; t < YRWI_MAX_TERMS; t++) P.sel_ninc[t] = P.sel_nexc[t] = 0;
    for (int li = 0; li < P.ninc + P.nexc; li++) {
      const ListRec* R = li < P.ninc ? P.linc[li] : P.lexc[li - P.ninc];
      if (!R || P.sel_uid.empty()) continue;
      SelCount c{};
      c.L = chain_list(R);
      c.sel = d_all + aoff[i];
      c.nsel = (int64_t)P.sel_uid.size();
      c.out = d_cnt + (int64_t)jobs.size();
      jobs.push_back(c);
      who.push_back({qs[i], li < P.ninc ? li : YRWI_MAX_TERMS + (li - P.ninc)});
    }
  }
  if (jobs.empty()) return 0;
  SelCount* d_jobs = arena_alloc<SelCount>(L, (int64_t)jobs.size());
  if (!d_jobs) return L->fail(YRWI_E_NOMEM, "arena");
  if (upload(L, d_all, all, d_jobs, jobs)) return YRWI_E_HIP;
  if (launch_sel_count(d_jobs, (int32_t)jobs.size(), L->stream)) return L->fail(YRWI_E_HIP, "selection count launch");
  const uint8_t* cb = readback(L, &L->down_stage, d_cnt, (int64_t)jobs.size(), 8, 8);
  if (!cb) return YRWI_E_HIP;
  HIPCHK(L, lane_sync(L));
  for (size_t j = 0; j < jobs.size(); j++) {
    int64_t c;
    std::memcpy(&c, cb + 8 * j, 8);
    Plan& P = plans[who[j].first];
    if (who[j].second < YRWI_MAX_TERMS) P.sel_ninc[who[j].second] = c;
    else P.sel_nexc[who[j].second - YRWI_MAX_TERMS] = c;
  }
  return 0;
}

// plan_finish for a batch: global term sizes from one exchange of the local
// sizes of the batch's distinct terms (sharded), or the local sizes (one context).
static int plan_batch(Lane* L, std::vector<Plan>& plans) {
  // a query with a url selection sees its lists restricted to it (resolve_selections)
  auto inc_n = [](const Plan& P, int i) -> int64_t { return P.has_sel ? P.sel_ninc[i] : P.linc[i] ? P.linc[i]->n : 0; };
  auto exc_n = [](const Plan& P, int i) -> int64_t { return P.has_sel ? P.sel_nexc[i] : P.lexc[i] ? P.lexc[i]->n : 0; };
  if (!L->sharded) {  // one context: its own sizes are the global ones
    for (Plan& P : plans) {
      int64_t gi[YRWI_MAX_TERMS], ge[YRWI_MAX_TERMS];
      for (int i = 0; i < P.ninc; i++) P.inc_allbm[i] = !P.has_sel && P.linc[i] && P.linc[i]->bm;
      for (int i = 0; i < P.ninc; i++) gi[i] = inc_n(P, i);
      for (int i = 0; i < P.nexc; i++) ge[i] = exc_n(P, i);
      plan_finish(&P, gi, ge);
    }
    return 0;
  }
  // every slot carries size * 128 + (this shard's list has a url-id bitmap): the
  // sum over the shards is the global size * 128 + the shards with a bitmap (< 128)
  std::unordered_map<KeyT, size_t, KeyHash> slot;
  std::vector<int64_t> sz;
  auto slot_of = [&](const KeyT& k, const ListRec* l) {
    auto it = slot.find(k);
    if (it != slot.end()) return it->second;
    slot.emplace(k, sz.size());
    sz.push_back(l ? l->n * 128 + (l->bm ? 1 : 0) : 0);
    return sz.size() - 1;
  };
  auto own_slot = [&](int64_t n) {  // a selection query's restricted size: a slot of its own
    sz.push_back(n * 128);
    return sz.size() - 1;
  };
  // first-appearance order over the batch's queries: identical on every rank
  std::vector<std::array<size_t, 2 * YRWI_MAX_TERMS>> idx(plans.size());
  for (size_t q = 0; q < plans.size(); q++) {
    Plan& P = plans[q];
    for (int i = 0; i < P.ninc; i++)
      idx[q][(size_t)i] = P.has_sel ? own_slot(inc_n(P, i)) : slot_of(P.inc[i], P.linc[i]);
    for (int i = 0; i < P.nexc; i++)
      idx[q][(size_t)(YRWI_MAX_TERMS + i)] = P.has_sel ? own_slot(exc_n(P, i)) : slot_of(P.exc[i], P.lexc[i]);
  }
  if (int rc = allsum_host(L, sz)) return rc;
  for (size_t q = 0; q < plans.size(); q++) {
    Plan& P = plans[q];
    int64_t gi[YRWI_MAX_TERMS], ge[YRWI_MAX_TERMS];
    for (int i = 0; i < P.ninc; i++) {
      const int64_t v = sz[idx[q][(size_t)i]];
      gi[i] = v >> 7;
      P.inc_allbm[i] = !P.has_sel && (v & 127) == L->world;
    }
    for (int i = 0; i < P.nexc; i++) ge[i] = sz[idx[q][(size_t)(YRWI_MAX_TERMS + i)]] >> 7;
    plan_finish(&P, gi, ge);
  }
  return 0;
}

// joinConstructive dispatch (ReferenceContainer.java:406-416); returns JoinMode
static int32_t dispatch_mode(int64_t n1, int64_t n2) {
  int32_t s1 = (int32_t)n1, s2 = (int32_t)n2;
  int32_t high = s1 > s2 ? s1 : s2, low = s1 > s2 ? s2 : s1;
  int32_t steps_enum = mul32(10, add32(add32(high, low), -1));
  int32_t steps_test = mul32(mul32(12, log2j(high)), low);
  if (steps_enum > steps_test) return s1 < s2 ? JM_TEST_LARGE_B : JM_TEST_LARGE_A;
  return JM_ENUM;
}

static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// algorithmic bytes of one join step
static int64_t step_bytes(int32_t mode, int64_t na, int64_t nb) {
  if (mode == JM_ENUM) return 12 * (na + nb);
  int64_t ns = std::min(na, nb), nl = std::max(na, nb);
  if (ns <= 0) return 0;  // by test with an empty smaller side: nothing is probed
  int64_t lg = 0;
  while ((ns << lg) < nl) lg++;  // ceil(log2(nl/ns))
  return 12 * (ns + std::min(nl, ns * (lg + 1)));
}

// bytes a join job's kernel loads (yrwi_stats.bytes_alg_capped): merge tiles
// stream both sides' 4-B url ids; a bitmap probe reads the smaller side's ids and
// one 16-B bitmap word per id; a range probe the ids and the larger list's range,
// or a 128-B leaf line per id, whichever is less (layout_jobs has set J.algo)
static int64_t loaded_bytes(const JoinQ& J) {
  const int64_t ns = std::min(J.A.n, J.B.n), nl = std::max(J.A.n, J.B.n);
  if (J.algo == JA_MERGE) return 4 * (ns + nl);
  if (J.algo == JA_BMAND) return (J.bm3 ? 48 : 32) * J.bm_words;  // every bitmap's 16-B units
  const bool bm = (J.small_is_A ? J.B.bm : J.A.bm) != nullptr;
  return bm ? 20 * ns : 4 * ns + std::min(4 * nl, 128 * ns);
}

struct Timing {
  // per join step: before k_join, between k_join and k_probe, after k_probe
  std::vector<std::array<hipEvent_t, 3>> kjoin;
  std::vector<std::array<hipEvent_t, 2>> kexcl;  // around each exclusion step's k_probe
  std::vector<std::array<hipEvent_t, 2>> kcompact;  // around each k_compact launch
  std::vector<std::array<hipEvent_t, 2>> kreduce;   // around each k_reduce + k_shard_fin
  std::vector<std::array<hipEvent_t, 2>> kscore;    // around each pass's k_score launches
  std::vector<std::array<hipEvent_t, 2>> kchain;    // around each chained step's k_chain_part .. k_scan_tiles
  // around every group of back-to-back kernel launches of the batch (no host
  // synchronisation inside a span): their sum is the batch's kernel time
  std::vector<std::array<hipEvent_t, 2>> spans;
  hipEvent_t t0 = nullptr, tj = nullptr, tn = nullptr, ts = nullptr;
};

static hipEvent_t span_open(Lane* L, Timing* tm) {
  if (!tm) return nullptr;
  hipEvent_t e = L->event();
  hipEventRecord(e, L->stream);
  return e;
}
static void span_close(Lane* L, Timing* tm, hipEvent_t b) {
  if (!tm) return;
  hipEvent_t e = L->event();
  hipEventRecord(e, L->stream);
  tm->spans.push_back({b, e});
}

// Give every job its algorithm and tile count, put merge jobs first and lay out
// the global tile index space: merge tiles [0, merge_tiles), probe tiles after.
static void layout_jobs(int64_t probe_ratio, int64_t nurls, std::vector<JoinQ>& jobs, std::vector<int>& owner,
                        std::vector<int64_t>& tile_base, int* nmerge, int64_t* merge_tiles, int64_t* tiles,
                        bool* long_tiles) {
  *long_tiles = false;
  std::vector<size_t> order(jobs.size());
  for (size_t i = 0; i < jobs.size(); i++) {
    JoinQ& J = jobs[i];
    // a counted-only join of two lists with bitmaps: popcounts of their words
    if (J.count_only && J.A.bm && J.B.bm && nurls > 0) {
      J.algo = JA_BMAND;
      J.small_is_A = 1;
      J.ptile = BMAND_WORDS;
      J.bm_words = bm_units(nurls);
      J.ntiles = ceil_div(J.bm_words, BMAND_WORDS);
      J.chain_bm = nullptr;
      order[i] = i;
      continue;
    }
    // a sparse list's bitmap (below 1/64 of the url ids: k_chain's tests and the
    // selections use it) does not take a join: its probes search the list, where
    // a tile's staged range costs less than a bitmap line per key
    if (J.A.bm && J.A.n * 64 < nurls) J.A.bm = nullptr;
    if (J.B.bm && J.B.n * 64 < nurls) J.B.bm = nullptr;
    const int64_t ns = std::min(J.A.n, J.B.n), nl = std::max(J.A.n, J.B.n);
    J.small_is_A = J.A.n <= J.B.n;
    // skewed sizes: probe the large list; a large list with a url-id bitmap is
    // probed at any ratio (the small side's ids stream, the bitmap stays in L2)
    const bool bm = (J.small_is_A ? J.B.bm : J.A.bm) != nullptr;
    J.algo = (bm || nl > probe_ratio * ns) ? JA_PROBE : JA_MERGE;
    // long bitmap tiles only where no record is gathered per match (a deferred
    // step writes sources, an exclusion marks): a final step's compaction keeps
    // its band order per 1024-id tile (C2 k_compact 220 -> 236 us with 2048)
    // A chained probe job whose first later include list has a bitmap (J.chain_bm,
    // set by the caller) tests it inside k_probe -- a bitmap probe on BM_TILE
    // tiles (the long tiles' registers leave no room for it), a range probe on its
    // usual tiles; merge jobs leave it to k_chain.
    if (J.algo == JA_MERGE) J.chain_bm = nullptr;
    const bool light = J.out_tup != nullptr || J.mode == JM_MARK || (J.chained && !J.chain_bm);
    J.ptile = bm ? (light && ns >= BM_LARGE_MIN ? KPT_LARGE * PROBE_TILE : BM_TILE) : PROBE_TILE;
    if (J.ptile == KPT_LARGE * PROBE_TILE) *long_tiles = true;
    J.ntiles = J.algo == JA_MERGE ? ceil_div(J.A.n + J.B.n, JOIN_TILE) : ceil_div(ns, J.ptile);
    order[i] = i;
  }
  // Within each algorithm, jobs that share their larger list run back to back:
  // queries sample terms by df, so the big lists recur across a batch, and
  // consecutive tiles over the same list hit in L2 / MALL instead of HBM.  Job
  // order only changes the schedule (every job owns its output slots).
  auto big = [&](const JoinQ& J) { return (uintptr_t)(J.A.n >= J.B.n ? J.A.uid : J.B.uid); };
  auto small = [&](const JoinQ& J) { return (uintptr_t)(J.A.n >= J.B.n ? J.B.uid : J.A.uid); };
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    const JoinQ &x = jobs[a], &y = jobs[b];
    if (x.algo != y.algo) return x.algo < y.algo;
    if (big(x) != big(y)) return big(x) < big(y);
    return small(x) < small(y);
  });
  std::vector<JoinQ> js;
  std::vector<int> ow;
  tile_base.clear();
  *nmerge = 0;
  *merge_tiles = 0;
  *tiles = 0;
  for (size_t i : order) {
    JoinQ J = jobs[i];
    J.tile_base = *tiles;
    tile_base.push_back(*tiles);
    *tiles += J.ntiles;
    if (J.algo == JA_MERGE) { (*nmerge)++; *merge_tiles = *tiles; }
    js.push_back(J);
    if (!owner.empty()) ow.push_back(owner[i]);
  }
  jobs.swap(js);
  if (!owner.empty()) owner.swap(ow);
}

static int64_t now_ns();

// band-major compaction schedule of a step's tiles (BandOrder, k_order_hist /
// k_order_scatter):
// scratch for the tile keys and the order; job order when disabled
static BandOrder band_order(Lane* ctx, int64_t tiles, int64_t merge_tiles, bool compact) {
  BandOrder bo;
  if (tiles <= 0 || tiles > INT32_MAX) return bo;
  bo.tile_job = arena_alloc<int32_t>(ctx, tiles);
  if (!ctx->band_order || tiles <= 1 || !bo.tile_job) return bo;
  bo.hist = arena_alloc<int32_t>(ctx, (int64_t)ORDER_HIST_SLICES * 4096);
  if (compact) {
    bo.key = arena_alloc<uint32_t>(ctx, tiles);
    bo.perm = arena_alloc<int2>(ctx, tiles);
  }
  if (tiles - merge_tiles > 1) {
    bo.pkey = arena_alloc<uint32_t>(ctx, tiles - merge_tiles);
    bo.pperm = arena_alloc<int2>(ctx, tiles - merge_tiles);
  }
  if (!bo.hist || (compact && (!bo.key || !bo.perm)) || (bo.pkey && !bo.pperm)) {
    bo.key = bo.pkey = nullptr;
    return bo;
  }
  int bits = 0;  // url ids < 2^bits; 2^12 bands for compaction, 2^4 for the probe
  while (bits < 32 && ((int64_t)1 << bits) < ctx->nurls) bits++;
  bo.shift = std::max(0, bits - 12);
  bo.pshift = std::max(0, bits - 4);
  return bo;
}

// A chained step whose compaction waits for the fold's dispatch modes (k_chain
// counts the intersections they depend on): what launch_compact needs.
struct PendingCompact {
  bool active = false;
  JoinQ* d_jobs = nullptr;
  int64_t* d_tb = nullptr;
  int nj = 0;
  int64_t tiles = 0;
  uint2* d_pairs = nullptr;
  uint32_t* d_puid = nullptr;
  int64_t* d_src = nullptr;
  int32_t* d_cnt = nullptr;
  int64_t* d_off = nullptr;
  BandOrder bo;
  int sum = 0;  // jobs with normalisation pieces (k_compact_sum): 0 none, 1 all, 2 some
  std::vector<std::array<int64_t, CHAIN_LVL>> level;  // per job (layout order): k_chain's level counts
};

// One fold step's join jobs: layout, launch, joined sizes back to the plans.
// chq (indexed by plan): the ChainQ of every chained query; a step with chained
// jobs runs k_chain and leaves its compaction to the caller (pend).
static int run_join_jobs(Lane* ctx, std::vector<Plan>& plans, std::vector<JoinQ>& jobs, std::vector<int>& owner,
                         yrwi_stats* st, Timing* tm, const std::vector<ChainQ>* chq = nullptr,
                         PendingCompact* pend = nullptr) {
  std::vector<int64_t> tile_base;
  int nmerge;
  int64_t merge_tiles, tiles;
  bool long_tiles;
  if (chq)  // candidates for the probe's own test of the first later include (layout_jobs)
    for (size_t j = 0; j < jobs.size(); j++) {
      const ChainQ& Cq = (*chq)[(size_t)owner[j]];
      jobs[j].chain_bm = jobs[j].chained && Cq.pos0 == 0 && Cq.ninc >= 1 ? Cq.l[0].bm : nullptr;
    }
  layout_jobs(ctx->probe_ratio, ctx->nurls, jobs, owner, tile_base, &nmerge, &merge_tiles, &tiles, &long_tiles);
  const int nj = (int)jobs.size();
  if (st)
    for (const JoinQ& J : jobs) {  // §8(d) K of the step as the reference dispatches it
      const int64_t K = step_bytes(J.mode, J.A.n, J.B.n), loaded = loaded_bytes(J);
      (J.algo == JA_MERGE ? st->bytes_join : st->bytes_probe) += K;
      (J.algo == JA_MERGE ? st->bytes_join_capped : st->bytes_probe_capped) += std::min(K, loaded);
      if (J.algo != JA_MERGE) st->bytes_probe_loaded += loaded;
      st->bytes_alg_capped += std::min(K, loaded);
    }
  bool chain = false;
  if (chq)
    for (int j = 0; j < nj; j++) chain |= jobs[(size_t)j].chained != 0;
  // joined sizes (and chained jobs' level counts) land in pinned host memory:
  // k_scan_tiles writes them through its device address (no copy engine), the host
  // reads them after the step's sync
  const size_t land_words = (size_t)nj * (chain ? 1 + CHAIN_LVL : 1);
  uint8_t* land = stage_reserve(ctx, &ctx->down_stage, land_words * sizeof(int64_t), true);
  if (!land) return YRWI_E_HIP;
  int64_t* d_mout = nullptr;
  HIPCHK(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&d_mout), land, 0));
  // pair runs: a job matches at most min(nA, nB) postings (both sides strictly
  // ascending); merge tiles bound theirs by min(na, nb + 1), at most one more per tile
  int64_t npairs = 0;
  for (int j = 0; j < nj; j++) {
    JoinQ& J = jobs[(size_t)j];
    J.m_out = d_mout + j;
    J.pair_base = npairs;
    if (!J.count_only) npairs += std::min(J.A.n, J.B.n) + (J.algo == JA_MERGE ? J.ntiles : 0);
  }
  JoinQ* d_jobs = arena_alloc<JoinQ>(ctx, nj);
  int64_t* d_tb = arena_alloc<int64_t>(ctx, nj);
  TileDesc* d_split = arena_alloc<TileDesc>(ctx, merge_tiles);
  ProbeDesc* d_pdesc = arena_alloc<ProbeDesc>(ctx, tiles - merge_tiles);
  // bitmap-probe tiles' short descriptors, in tile order and in k_probe's order
  BmFast* d_fast = arena_alloc<BmFast>(ctx, tiles - merge_tiles);
  BmFast* d_fast_perm = arena_alloc<BmFast>(ctx, tiles - merge_tiles);
  uint2* d_pairs = arena_alloc<uint2>(ctx, npairs);
  uint32_t* d_puid = arena_alloc<uint32_t>(ctx, npairs);
  int64_t* d_src = arena_alloc<int64_t>(ctx, tiles);
  int32_t* d_cnt = arena_alloc<int32_t>(ctx, tiles);
  int64_t* d_off = arena_alloc<int64_t>(ctx, tiles);
  if (!d_jobs || !d_tb || !d_split || !d_pdesc || !d_fast || !d_fast_perm || !d_pairs || !d_puid || !d_src ||
      !d_cnt || !d_off)
    return ctx->fail(YRWI_E_NOMEM, "arena");
  // the queries' last steps that summarise their containers as they compact them:
  // one ChunkSum per tile of the step, the job's run from its first tile
  auto sum_mode = [&]() {
    bool any = false, all = true;
    for (const JoinQ& J : jobs) {
      if (J.count_only) continue;
      any |= J.psum != nullptr;
      all &= J.psum != nullptr;
    }
    return any ? (all ? 1 : 2) : 0;
  };
  bool any_want = false;
  for (const JoinQ& J : jobs) any_want |= J.want_sum != 0;
  if (any_want) {
    ChunkSum* d_psum = arena_alloc<ChunkSum>(ctx, tiles);
    if (!d_psum) return ctx->fail(YRWI_E_NOMEM, "arena");
    for (int j = 0; j < nj; j++)
      if (jobs[(size_t)j].want_sum) jobs[(size_t)j].psum = d_psum + tile_base[(size_t)j];
  }
  const int sum = sum_mode();
  // chained jobs: their ChainQ (level counts into the landing buffer, the later
  // include lists' rows in slot-indexed arrays beside the pairs), per-tile level
  // counts and the list ranges of k_chain_part
  int32_t* d_lvl = nullptr;
  ProbeDesc* d_crange = nullptr;
  std::vector<ChainQ> cq;
  ChainQ* d_cq = nullptr;
  std::vector<int2> cgrp;  // chain groups: runs of up to CHAIN_GMAX merge tiles of one chained job (k_chain)
  int2* d_cgrp = nullptr;
  if (chain) {
    // a group holds about 640 expected matches (independent lists: nA nB / nurls
    // per job), so a workgroup tests close to one round of 768
    for (int j = 0; j < nj; j++) {
      const JoinQ& J = jobs[(size_t)j];
      if (!J.chained || J.ntiles <= 0) continue;
      double per_tile = (double)J.A.n * (double)J.B.n / (double)std::max<int64_t>(1, ctx->nurls) /
                        (double)J.ntiles;
      const ChainQ& Cq = (*chq)[(size_t)owner[(size_t)j]];
      if (J.chain_bm)  // the probe already thinned the matches by the first later include
        per_tile *= std::min(1.0, (double)Cq.l[0].n / (double)std::max<int64_t>(1, ctx->nurls));
      const int G = (int)std::max(1.0, std::min((double)CHAIN_GMAX, 640.0 / std::max(1.0, per_tile)));
      for (int64_t t = 0; t < J.ntiles; t += G)
        cgrp.push_back(make_int2((int32_t)(tile_base[(size_t)j] + t), (int32_t)std::min<int64_t>(G, J.ntiles - t)));
    }
    d_lvl = arena_alloc<int32_t>(ctx, tiles * CHAIN_LVL);
    d_crange = arena_alloc<ProbeDesc>(ctx, (int64_t)cgrp.size() * CHAIN_MAXL);
    d_cgrp = arena_alloc<int2>(ctx, (int64_t)cgrp.size());
    d_cq = arena_alloc<ChainQ>(ctx, nj);
    if (!d_lvl || !d_crange || !d_cgrp || !d_cq) return ctx->fail(YRWI_E_NOMEM, "arena");
    int maxi = 0;
    for (int j = 0; j < nj; j++)
      if (jobs[(size_t)j].chained) maxi = std::max(maxi, (*chq)[(size_t)owner[(size_t)j]].npos);
    int32_t* d_tup[CHAIN_MAXI] = {nullptr, nullptr};  // rows in the later include lists, indexed like d_pairs
    for (int l = 0; l < maxi; l++)
      if (!(d_tup[l] = arena_alloc<int32_t>(ctx, npairs))) return ctx->fail(YRWI_E_NOMEM, "arena");
    for (int j = 0; j < nj; j++) {
      JoinQ& J = jobs[(size_t)j];
      const int pq = owner[(size_t)j];
      if (!J.chained) continue;  // (a count-first fold's counted job is not)
      ChainQ C = (*chq)[(size_t)pq];
      C.level = d_mout + nj + (int64_t)j * CHAIN_LVL;
      for (int l = 0; l < CHAIN_MAXI; l++) C.tup[l] = l < C.npos ? d_tup[l] : nullptr;
      // a bitmap probe tests the first later include list itself when that list
      // has a bitmap (no selection before it): only its survivors reach k_chain
      C.pre = J.chain_bm != nullptr ? 1 : 0;  // (layout_jobs kept it for bitmap probes only)
      J.chain_tup0 = C.pre ? C.tup[0] : nullptr;
      J.chain_fill = C.pre && C.ninc == 1 ? 2 : 0;
      J.chain = d_cq + (int64_t)cq.size();
      cq.push_back(C);
    }
  }
  if (chain ? upload(ctx, d_jobs, jobs, d_tb, tile_base, d_cq, cq, d_cgrp, cgrp)
            : upload(ctx, d_jobs, jobs, d_tb, tile_base))
    return YRWI_E_HIP;
  hipEvent_t e0 = tm ? ctx->event() : nullptr, em = tm ? ctx->event() : nullptr, e1 = tm ? ctx->event() : nullptr;
  hipEvent_t c0 = tm ? ctx->event() : nullptr, c1 = tm ? ctx->event() : nullptr;
  hipEvent_t sp = span_open(ctx, tm);
  const BandOrder bo = band_order(ctx, tiles, merge_tiles, true);
  if (launch_join_step(d_jobs, d_tb, nj, nmerge, merge_tiles, tiles, d_split, d_pdesc, d_pairs, d_puid, d_src, d_cnt, d_off,
                       false, long_tiles, bo, ctx->stream, e0, em, e1, c0, c1, chain, d_lvl, d_crange, d_cgrp,
                       (int64_t)cgrp.size(), d_fast, d_fast_perm, sum))
    return ctx->fail(YRWI_E_HIP, "join launch");
  if (tm) {
    tm->kjoin.push_back({e0, em, e1});
    // the span ends after k_scan_tiles (chained steps: compaction comes later)
    hipEvent_t se = ctx->event();
    hipEventRecord(se, ctx->stream);
    if (chain) {
      // c0 / c1 bracket k_chain alone; a step without chain groups launched none
      if (!cgrp.empty()) tm->kchain.push_back({c0, c1});
    } else {
      tm->kcompact.push_back({c0, c1});
    }
    tm->spans.push_back({sp, se});
  }
  if (st) {
    st->n_join_launches++;
    st->n_probe_dispatches += tiles > merge_tiles;
    st->n_chain_launches += chain && !cgrp.empty() ? 1 : 0;  // k_chain launches (timed in t_chain_ns)
  }
  std::vector<int64_t> mh((size_t)nj, 0);
  HIPCHK(ctx, lane_sync(ctx));
  std::memcpy(mh.data(), land, (size_t)nj * sizeof(int64_t));
  if (st)  // k_compact per joined row: pair + id read, the records it gathers (32 B, + 16 B of the joined
           // side for enumeration steps, + the deferred rows' sources and records), record + id written;
           // deferred output: A's sources read, sources + id written; chained: the rows of every list of
           // the fold (4 B each beyond the pair), the records of the fold (32 B + 16 B per enumeration step)
    for (int j = 0; j < nj; j++) {
      const JoinQ& J = jobs[(size_t)j];
      const int64_t atw = J.A.tup ? J.A.tw : 0;
      if (J.count_only) continue;
      if (J.chain) {
        const int64_t t = 2 + (*chq)[(size_t)owner[(size_t)j]].npos;
        st->bytes_compact += mh[(size_t)j] * (12 + 4 * (t - 2) + 32 + 24 * (t - 1) + 36);
        continue;
      }
      st->bytes_compact += mh[(size_t)j] * (J.out_tup ? 12 + 4 * atw + 4 + 4 * (int64_t)J.out_tw
                                                      : (J.mode == JM_ENUM ? 96 : 80) + 4 * atw +
                                                            (atw > 1 ? 24 * (atw - 1) : 0));
    }
  if (chain) {  // chained jobs' containers, sized by their survivors; the job table again for k_compact
    for (int j = 0; j < nj; j++) {
      JoinQ& J = jobs[(size_t)j];
      if (!J.chain) continue;
      J.out_uid = arena_alloc<uint32_t>(ctx, mh[(size_t)j]);
      J.out_feat = arena_alloc<uint64_t>(ctx, mh[(size_t)j] * FEAT_WORDS);
      if (!J.out_uid || !J.out_feat) return ctx->fail(YRWI_E_NOMEM, "arena");
    }
    if (upload(ctx, d_jobs, jobs)) return YRWI_E_HIP;
  }
  for (int j = 0; j < nj; j++) {
    Plan& P = plans[(size_t)owner[(size_t)j]];
    const JoinQ& J = jobs[(size_t)j];
    if (J.count_only) {
      (J.bm3 ? P.cf_count2 : P.cf_count) = mh[(size_t)j];
      continue;
    }
    P.cont = DList{nullptr, nullptr, nullptr, mh[(size_t)j], J.out_uid, J.out_feat, nullptr, J.out_tup,
                   J.out_tup ? J.out_tw : 0};
    P.pieces = J.psum;
    P.npieces = J.psum ? J.ntiles : 0;
  }
  if (chain && pend) {
    pend->active = true;
    pend->d_jobs = d_jobs;
    pend->d_tb = d_tb;
    pend->nj = nj;
    pend->tiles = tiles;
    pend->d_pairs = d_pairs;
    pend->d_puid = d_puid;
    pend->d_src = d_src;
    pend->d_cnt = d_cnt;
    pend->d_off = d_off;
    pend->bo = bo;
    pend->sum = sum;
    pend->level.assign((size_t)nj, {0, 0, 0, 0, 0});
    const int64_t* hl = reinterpret_cast<const int64_t*>(land) + nj;
    for (int j = 0; j < nj; j++)
      if (jobs[(size_t)j].chain)
        for (int l = 0; l < CHAIN_LVL; l++) pend->level[(size_t)j][(size_t)l] = hl[(int64_t)j * CHAIN_LVL + l];
  }
  return 0;
}

// exclusion (excludeContainers :373-388): mark container rows present in an exclude list
static int run_exclusion(Lane* ctx, std::vector<Plan>& plans, yrwi_stats* st, Timing* tm) {
  std::vector<JoinQ> jobs;
  std::vector<int> owner;
  std::vector<int64_t> tile_base;
  for (auto& P : plans) {
    P.removed = nullptr;
    if (P.empty || P.cont.n == 0 || P.excl.empty()) continue;
    P.removed = arena_alloc<uint8_t>(ctx, P.cont.n);
    if (!P.removed) return ctx->fail(YRWI_E_NOMEM, "arena");
    HIPCHK(ctx, hipMemsetAsync(P.removed, 0, (size_t)P.cont.n, ctx->stream));
    for (auto* E : P.excl) {
      JoinQ J{};
      J.A = P.cont;
      J.B = E->dl();
      J.mode = JM_MARK;
      J.maxd = YRWI_MAX_DISTANCE_ANY;
      J.removed = P.removed;
      if (st) st->bytes_alg += 12 * E->n;
      jobs.push_back(J);
    }
  }
  if (jobs.empty()) return 0;
  int nmerge;
  int64_t merge_tiles, tiles;
  bool long_tiles;
  layout_jobs(ctx->probe_ratio, ctx->nurls, jobs, owner, tile_base, &nmerge, &merge_tiles, &tiles, &long_tiles);
  const int nj = (int)jobs.size();
  if (st)
    for (const JoinQ& J : jobs) st->bytes_alg_capped += std::min<int64_t>(12 * J.B.n, loaded_bytes(J));
  JoinQ* d_jobs = arena_alloc<JoinQ>(ctx, nj);
  int64_t* d_tb = arena_alloc<int64_t>(ctx, nj);
  TileDesc* d_split = arena_alloc<TileDesc>(ctx, merge_tiles);
  ProbeDesc* d_pdesc = arena_alloc<ProbeDesc>(ctx, tiles - merge_tiles);
  if (!d_jobs || !d_tb || !d_split || !d_pdesc) return ctx->fail(YRWI_E_NOMEM, "arena");
  if (upload(ctx, d_jobs, jobs, d_tb, tile_base)) return YRWI_E_HIP;
  const BandOrder bo = band_order(ctx, tiles, merge_tiles, false);
  hipEvent_t sp = span_open(ctx, tm);
  hipEvent_t pm = tm ? ctx->event() : nullptr, p1 = tm ? ctx->event() : nullptr;
  if (launch_join_step(d_jobs, d_tb, nj, nmerge, merge_tiles, tiles, d_split, d_pdesc, nullptr, nullptr, nullptr, nullptr,
                       nullptr, true, long_tiles, bo,
                       ctx->stream, nullptr, pm, p1))
    return ctx->fail(YRWI_E_HIP, "exclude launch");
  span_close(ctx, tm, sp);
  if (tm) tm->kexcl.push_back({pm, p1});
  if (st) st->n_probe_dispatches += tiles > merge_tiles;
  return 0;
}

// Run the join/exclusion phase of all plans; leaves each plan's container in P.cont.
// Every fold step's dispatch (J3) is taken on the global sizes of its two
// containers: the next list's (Plan.seq_ng) and the accumulated container's,
// which after the first step is the sum over the shards of their joined rows
// (one exchange per step that some query continues past; none on one context).
static int run_join_phase(Lane* ctx, std::vector<Plan>& plans, yrwi_stats* st, Timing* tm) {
  const size_t nq = plans.size();
  std::vector<int64_t> acc_g(nq, 0);  // global size of each query's accumulated container
  for (size_t qi = 0; qi < nq; qi++) {
    Plan& P = plans[qi];
    if (P.empty) { P.cont = DList{nullptr, nullptr, nullptr, 0}; continue; }
    P.cont = P.seq[0]->dl();  // (a single list under a url selection: restricted below)
    acc_g[qi] = P.seq_ng[0];
  }
  constexpr bool defer = true;  // deferred multi-term folds (round 2): a step before the last writes sources only
  // Chained folds (ChainQ): every query with lists after its first join step --
  // later includes (t <= 4) and / or exclusions -- and no maxDistance filter.  The
  // decision rests on global facts only (fold length, exclusion terms in effect),
  // so every shard takes it alike.  YRWI_NO_CHAIN=1: the step-by-step fold.
  const char* nc = getenv("YRWI_NO_CHAIN");  // read per call: tests compare both paths in one process
  const bool chain_on = !(nc && atoi(nc));
  // YRWI_CHAIN_CF: 0 never count-first, 2 every 3-term chained fold (tests), default 1 (list 2 the smallest)
  const char* cfe = getenv("YRWI_CHAIN_CF");
  const int cf_mode = cfe ? atoi(cfe) : 1;
  std::vector<ChainQ> chq(nq);
  bool any_chain = false;
  // url selections (resolve_selections): their ids for this pass's kernels; a
  // single include list is restricted right here (k_sel_pick), a fold of two or
  // more chains the selection as its first test (ChainQ)
  std::vector<uint32_t*> dsel(nq, nullptr);
  std::vector<SelPick> picks;
  for (size_t qi = 0; qi < nq; qi++) {
    Plan& P = plans[qi];
    if (!P.has_sel || P.empty) continue;
    if (!P.sel_uid.empty()) {
      if (!(dsel[qi] = arena_alloc<uint32_t>(ctx, (int64_t)P.sel_uid.size()))) return ctx->fail(YRWI_E_NOMEM, "arena");
      if (upload(ctx, dsel[qi], P.sel_uid)) return YRWI_E_HIP;
    }
    if (P.seq.size() == 1) {  // ReferenceContainer.java:355-370: the one (restricted) container, rows as stored
      const int64_t m = P.sel_ninc[P.seq_term[0]];
      P.cont = DList{nullptr, nullptr, nullptr, 0};
      if (m == 0 || P.seq[0]->n == 0) continue;
      SelPick k{};
      k.L = chain_list(P.seq[0]);
      k.feat = P.seq[0]->feat;
      k.rows = P.seq[0]->rows;
      k.sel = dsel[qi];
      k.nsel = (int64_t)P.sel_uid.size();
      k.out_uid = arena_alloc<uint32_t>(ctx, m);
      k.out_feat = arena_alloc<uint64_t>(ctx, m * FEAT_WORDS);
      k.out_rows = arena_alloc<uint8_t>(ctx, m * YRWI_ROW_BYTES);
      if (!k.out_uid || !k.out_feat || !k.out_rows) return ctx->fail(YRWI_E_NOMEM, "arena");
      P.cont = DList{nullptr, nullptr, k.out_rows, m, k.out_uid, k.out_feat, nullptr, nullptr, 0};
      picks.push_back(k);
    }
  }
  if (!picks.empty()) {
    SelPick* d_pk = arena_alloc<SelPick>(ctx, (int64_t)picks.size());
    if (!d_pk) return ctx->fail(YRWI_E_NOMEM, "arena");
    if (upload(ctx, d_pk, picks)) return YRWI_E_HIP;
    if (launch_sel_pick(d_pk, (int32_t)picks.size(), ctx->stream)) return ctx->fail(YRWI_E_HIP, "selection launch");
  }
  for (size_t qi = 0; qi < nq; qi++) {
    Plan& P = plans[qi];
    P.chain = false;
    const int t = (int)P.seq.size(), ni = t - 2, ns = P.has_sel ? 1 : 0;
    const bool can = chain_on && defer && !P.empty && P.maxd >= 65535 && acc_g[qi] > 0 && t >= 2 &&
                     ni <= CHAIN_MAXI && ns + ni + P.nexcl_g > 0 && ns + ni + P.nexcl_g <= CHAIN_MAXL;
    if (P.has_sel && !P.empty && t >= 2 && !can)
      return ctx->fail(YRWI_E_UNSUPPORTED, "urlselection: a fold of more than four include terms or with a "
                                           "maxDistance filter");
    if (!can) continue;
    ChainQ& C = chq[qi];
    std::memset(&C, 0, sizeof(C));
    C.nl = 0;
    // Count-first (t = 3 whose list 2 is the smallest -- J2's int-wrapped keys put
    // big lists first: C3's 52 such queries make 85 of its 98 M first-step
    // matches): list 0 x list 1 is only counted (its size is step 1's dispatch),
    // the survivors are chained from list 2 (probing list 0, then testing list 1)
    // (t = 4 too: the chain's first test, list 1, leaves |list 0..2| -- step 2's
    // dispatch -- and list 3 follows)
    // (lists 0..2 with bitmaps on every shard -- the planning exchange decides it
    // alike on every rank -- so every shard counts by popcounts)
    P.cf3 = cf_mode != 0 && t == 4 && !ns && P.inc_allbm[P.seq_term[0]] && P.inc_allbm[P.seq_term[1]] &&
            P.inc_allbm[P.seq_term[2]] &&
            (cf_mode == 2 || (P.seq_ng[3] < P.seq_ng[0] && P.seq_ng[3] < P.seq_ng[1] && P.seq_ng[3] < P.seq_ng[2]));
    P.cf = !P.cf3 && cf_mode != 0 && (t == 3 || t == 4) && !ns &&
           (cf_mode == 2 || (P.seq_ng[2] < P.seq_ng[0] && P.seq_ng[2] < P.seq_ng[1]));
    if (ns)  // the selection first: its ids, no heads, no bitmap
      C.l[C.nl++] = ChainList{dsel[qi], nullptr, nullptr, (int64_t)P.sel_uid.size()};
    if (P.cf) {
      C.l[C.nl++] = chain_list(P.seq[1]);
      if (t == 4) C.l[C.nl++] = chain_list(P.seq[3]);
    } else if (P.cf3) {
      C.l[C.nl++] = chain_list(P.seq[1]);
      C.l[C.nl++] = chain_list(P.seq[2]);
    } else {
      for (int l = 0; l < ni; l++) C.l[C.nl++] = chain_list(P.seq[(size_t)l + 2]);
    }
    C.ninc = C.nl;
    C.pos0 = ns;
    C.npos = ni;
    C.perm = P.cf ? 1 : P.cf3 ? 2 : 0;
    for (const ListRec* E : P.excl) C.l[C.nl++] = chain_list(E);  // this shard's lists of the exclusion terms
    if (st)
      for (const ListRec* E : P.excl) st->bytes_alg += 12 * E->n;
    P.excl.clear();  // excluded inside k_chain: no marks, no exclusion step
    P.chain = true;
    any_chain = true;
  }
  // a query steps at s while it has a list left and its global container is not empty
  auto steps = [&](size_t qi, size_t s) {
    const Plan& P = plans[qi];
    return !P.empty && P.seq.size() > s + 1 && acc_g[qi] > 0 && !(P.chain && s > 0);
  };
  for (size_t s = 0;; s++) {
    std::vector<JoinQ> jobs;
    std::vector<int> owner;
    std::vector<FoldSrc> fold;
    std::vector<int> fold_job;
    std::vector<int> chain_q;  // chained queries with a job in this step (plan index)
    bool any = false, more = false;  // some query steps now / after this step (global decisions)
    for (size_t qi = 0; qi < nq; qi++) {
      if (!steps(qi, s)) continue;
      any = true;
      Plan& P = plans[qi];
      if (P.seq.size() > s + 2 && !P.chain) more = true;
      const DList B = P.seq[s + 1]->dl();
      if (P.chain) P.step_mode[s] = dispatch_mode(acc_g[qi], P.seq_ng[s + 1]);
      if (P.cont.n == 0 || B.n == 0) {  // nothing of this shard survives the step
        P.cont = DList{nullptr, nullptr, nullptr, 0};
        continue;
      }
      JoinQ J{};
      J.A = P.cont;
      J.B = B;
      J.mode = dispatch_mode(acc_g[qi], P.seq_ng[s + 1]);
      J.maxd = P.maxd;
      J.now_ms = P.now_ms;
      J.chained = P.chain ? 1 : 0;
      P.step_mode[s] = J.mode;
      if (P.cf || P.cf3) {  // count-first: list 0 x list 1 counted, the chained job probes list 2 (3) into list 0
        JoinQ K = J;
        K.chained = 0;
        K.count_only = 1;
        if (st) st->bytes_alg += step_bytes(K.mode, K.A.n, K.B.n);
        jobs.push_back(K);
        owner.push_back((int)qi);
        if (P.cf3) {  // and list 0 x list 1 x list 2 (a three-way popcount)
          K.bm3 = P.seq[2]->bm;
          jobs.push_back(K);
          owner.push_back((int)qi);
        }
        const DList L2 = P.seq[P.cf3 ? 3 : 2]->dl();
        if (L2.n == 0) {  // nothing of this shard survives (its count still goes in)
          P.cont = DList{nullptr, nullptr, nullptr, 0};
          continue;
        }
        J.A = L2;
        J.B = P.cont;
        J.mode = JM_ENUM;  // (the chained job's records are folded by fold_chain with the fold's modes)
      }
      int64_t cap = std::min(J.A.n, J.B.n);
      // a chained job's output is allocated once k_chain has counted its survivors
      // (run_join_jobs): its capacity bound min(nA, nB) is far above them
      J.out_uid = P.chain ? nullptr : arena_alloc<uint32_t>(ctx, cap);
      // A step before the fold's last keeps its rows deferred (the rows of lists
      // 0..s+1 they join, no records): the next step joins on url ids alone, and
      // only the last step gathers and folds the records of the rows that survive.
      // A maxDistance filter needs every step's joined features: materialised.
      // A chained query's first step is its only one.
      const bool last = P.seq.size() == s + 2 || P.chain;
      if (!last && defer && P.maxd >= 65535) {
        J.out_tw = (int32_t)s + 2;
        J.out_tup = arena_alloc<int32_t>(ctx, cap * J.out_tw);
        if (!J.out_tup) return ctx->fail(YRWI_E_NOMEM, "arena");
      } else {
        J.out_feat = P.chain ? nullptr : arena_alloc<uint64_t>(ctx, cap * FEAT_WORDS);
        if (!J.out_feat && !P.chain) return ctx->fail(YRWI_E_NOMEM, "arena");
        // the container the rank phase reads: summarised by the compaction unless
        // exclusion marks (run_exclusion, after this) or host counts need a pass over
        // it.  Not a chained fold with exclusions inside the chain: its survivors are
        // sparse in their tiles, and k_compact, four tiles per workgroup, packs them
        // (C3 1.23 -> 1.37 ms/step through k_compact_sum); the chained folds without
        // take the pieces (C4 9.59-9.69 -> 9.24-9.26 ms/step against pieces only for
        // those averaging 64 survivors per tile, 9.47-9.52 at 16)
        const bool chain_excl = P.chain && chq[qi].nl > chq[qi].ninc;
        J.want_sum = last && P.excl.empty() && !chain_excl && P.prof.coeff_authority <= 12 ? 1 : 0;
        if (P.chain) {
          chain_q.push_back((int)qi);
        } else if (J.A.tup) {
          FoldSrc F{};
          for (int l = 0; l < J.A.tw; l++) {
            F.feat[l] = P.seq[(size_t)l]->feat;
            F.j5[l] = P.seq[(size_t)l]->j5;
          }
          for (size_t t = 0; t < s; t++) F.mode[t] = P.step_mode[t];
          fold.push_back(F);
          fold_job.push_back((int)jobs.size());
        }
      }
      if (!J.out_uid && !P.chain) return ctx->fail(YRWI_E_NOMEM, "arena");
      if (st) {
        st->bytes_alg += step_bytes(J.mode, J.A.n, J.B.n);
        if (J.mode == JM_ENUM) st->n_enum_steps++; else st->n_test_steps++;
      }
      jobs.push_back(J);
      owner.push_back((int)qi);
    }
    if (!any) break;
    if (!fold.empty()) {  // the fold programs of the jobs whose A is deferred
      FoldSrc* d_fold = arena_alloc<FoldSrc>(ctx, (int64_t)fold.size());
      if (!d_fold) return ctx->fail(YRWI_E_NOMEM, "arena");
      if (upload(ctx, d_fold, fold)) return YRWI_E_HIP;
      for (size_t f = 0; f < fold.size(); f++) jobs[(size_t)fold_job[f]].fold = d_fold + f;
    }
    // chained queries: their fold programs are written once the modes are known
    FoldSrc* d_cfold = nullptr;
    std::vector<int> cfold_of(nq, -1);
    if (!chain_q.empty()) {
      d_cfold = arena_alloc<FoldSrc>(ctx, (int64_t)chain_q.size());
      if (!d_cfold) return ctx->fail(YRWI_E_NOMEM, "arena");
      for (size_t k = 0; k < chain_q.size(); k++) cfold_of[(size_t)chain_q[k]] = (int)k;
      for (size_t j = 0; j < jobs.size(); j++)
        if (cfold_of[(size_t)owner[j]] >= 0) jobs[j].fold = d_cfold + cfold_of[(size_t)owner[j]];
    }
    PendingCompact pend;
    if (!jobs.empty())
      if (int rc = run_join_jobs(ctx, plans, jobs, owner, st, tm, any_chain ? &chq : nullptr, &pend)) return rc;
    if (s == 0 && any_chain) {
      // the fold's later steps: their dispatch (J3) from the GLOBAL intersection
      // sizes (k_chain's level counts summed over the shards), then the records
      std::vector<int> cqs;
      for (size_t qi = 0; qi < nq; qi++)
        if (plans[qi].chain && steps(qi, 0)) cqs.push_back((int)qi);
      std::vector<int> job_of(nq, -1);
      for (size_t j = 0; j < jobs.size(); j++)
        if (!jobs[j].count_only) job_of[(size_t)owner[j]] = (int)j;
      std::vector<int64_t> v(cqs.size() * 2, 0);
      for (size_t k = 0; k < cqs.size(); k++) {
        const int j = job_of[(size_t)cqs[k]];
        if (plans[(size_t)cqs[k]].cf3) {  // from list 3: both sizes counted apart
          v[2 * k] = plans[(size_t)cqs[k]].cf_count;
          v[2 * k + 1] = plans[(size_t)cqs[k]].cf_count2;
        } else if (plans[(size_t)cqs[k]].cf) {  // count-first: |list 0 x list 1| counted apart, then |list 0..2|
          v[2 * k] = plans[(size_t)cqs[k]].cf_count;
          if (j >= 0 && pend.active) v[2 * k + 1] = pend.level[(size_t)j][1];
        } else if (j >= 0 && pend.active) {  // the intersection sizes after the selection (if any) and include 2
          const int o = chq[(size_t)cqs[k]].pos0;
          v[2 * k] = pend.level[(size_t)j][(size_t)o];
          v[2 * k + 1] = pend.level[(size_t)j][(size_t)o + 1];
        }
      }
      std::vector<int64_t> loc = v;
      if (int rc = allsum_host(ctx, v)) return rc;
      std::vector<FoldSrc> cf(chain_q.size());
      for (size_t k = 0; k < cqs.size(); k++) {
        Plan& P = plans[(size_t)cqs[k]];
        const int t = (int)P.seq.size();
        if (t >= 3) P.step_mode[1] = dispatch_mode(v[2 * k], P.seq_ng[2]);
        if (t >= 4) P.step_mode[2] = dispatch_mode(v[2 * k + 1], P.seq_ng[3]);
        if (st) {  // the later steps' K (local sizes), charged min(K, the bytes the chain tests load for them)
          for (int l = 2; l < t; l++) {
            const int64_t acc = loc[2 * k + (size_t)(l - 2)], n = P.seq[(size_t)l]->n;
            const int32_t m = P.step_mode[l - 1];
            const int64_t K = step_bytes(m, acc, n);
            const int64_t loaded = P.seq[(size_t)l]->bm ? 20 * acc : 4 * acc + std::min(4 * n, 128 * acc);
            st->bytes_alg += K;
            st->bytes_chain += std::min(K, loaded);
            st->bytes_alg_capped += std::min(K, loaded);
            if (m == JM_ENUM) st->n_enum_steps++; else st->n_test_steps++;
          }
        }
        const int f = cfold_of[(size_t)cqs[k]];
        if (f < 0) continue;  // no job of this query on this shard
        FoldSrc& F = cf[(size_t)f];
        for (int l = 0; l < t; l++) {
          F.feat[l] = P.seq[(size_t)l]->feat;
          F.j5[l] = P.seq[(size_t)l]->j5;
        }
        for (int l = 0; l + 1 < t; l++) F.mode[l] = P.step_mode[l];
      }
      if (!cf.empty() && upload(ctx, d_cfold, cf)) return YRWI_E_HIP;
      if (pend.active) {
        hipEvent_t c0 = tm ? ctx->event() : nullptr, c1 = tm ? ctx->event() : nullptr;
        if (c0) hipEventRecord(c0, ctx->stream);
        if (launch_compact(pend.d_jobs, pend.d_tb, pend.nj, pend.tiles, pend.d_pairs, pend.d_puid, pend.d_src,
                           pend.d_cnt, pend.d_off, pend.bo, true, ctx->stream, pend.sum))
          return ctx->fail(YRWI_E_HIP, "compact launch");
        if (c1) {
          hipEventRecord(c1, ctx->stream);
          tm->kcompact.push_back({c0, c1});
          tm->spans.push_back({c0, c1});
        }
      }
      if (st) {  // exclusions of chained queries: the bytes k_chain loads for them
        for (size_t k = 0; k < cqs.size(); k++) {
          const int j = job_of[(size_t)cqs[k]];
          const ChainQ& C = chq[(size_t)cqs[k]];
          const int64_t pre = (j >= 0 && pend.active) ? pend.level[(size_t)j][(size_t)C.ninc] : 0;
          for (int l = C.ninc; l < C.nl; l++) {
            const int64_t b = std::min<int64_t>(12 * C.l[l].n, C.l[l].bm ? 20 * pre
                                                                         : 4 * pre + std::min(4 * C.l[l].n, 128 * pre));
            st->bytes_alg_capped += b;
            st->bytes_chain += b;
          }
        }
      }
    } else if (pend.active) {
      return ctx->fail(YRWI_E_HIP, "chained step outside the first fold step");
    }
    if (!more) break;
    // the accumulated containers' global sizes decide the next step's dispatch
    std::vector<int64_t> v(nq, 0);
    std::vector<char> stepped(nq, 0);
    for (size_t qi = 0; qi < nq; qi++)
      if (steps(qi, s)) { v[qi] = plans[qi].cont.n; stepped[qi] = 1; }
    if (int rc = allsum_host(ctx, v)) return rc;
    for (size_t qi = 0; qi < nq; qi++)
      if (stepped[qi]) acc_g[qi] = v[qi];
  }
  return run_exclusion(ctx, plans, st, tm);
}

// Global host counts for authority (ReferenceOrder.java:176-216) across url-hash
// shards: (query, host, count) messages to the host's owner rank, summed there,
// totals sent back; the per-query max count is all-reduced.  Collective.
static int exchange_host_counts(Lane* ctx, int nq, int64_t nslots, const std::vector<int64_t>& slot_base,
                                uint64_t* d_hkeys, uint32_t* d_hcnt, ShardSum* d_ss) {
  const int W = ctx->world, me = ctx->rank;
  uint32_t* d_ocnt = arena_alloc<uint32_t>(ctx, W);
  uint32_t* d_M = arena_alloc<uint32_t>(ctx, (int64_t)W * W);
  int64_t* d_sb = arena_alloc<int64_t>(ctx, nq + 1);
  int32_t* d_gmax = arena_alloc<int32_t>(ctx, nq);
  if (!d_ocnt || !d_M || !d_sb || !d_gmax) return ctx->fail(YRWI_E_NOMEM, "arena");
  HIPCHK(ctx, hipMemsetAsync(d_ocnt, 0, W * 4, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync(d_gmax, 0, nq * 4, ctx->stream));
  if (upload(ctx, d_sb, slot_base)) return YRWI_E_HIP;
  const uint64_t* hkey = ctx->host_ids ? ctx->host_key : nullptr;  // tables of dense host ids (run_rank_phase)
  if (launch_host_count(d_hkeys, nslots, W, d_ocnt, ctx->stream, hkey)) return ctx->fail(YRWI_E_HIP, "host count");
  if (int rc = coll_allgather(ctx, d_ocnt, d_M, (size_t)W * 4)) return rc;
  const uint8_t* hm = readback(ctx, &ctx->down_stage, d_M, (int64_t)W * W, 4, 4);
  if (!hm) return YRWI_E_HIP;
  HIPCHK(ctx, lane_sync(ctx));
  std::vector<uint32_t> M((size_t)W * W);
  std::memcpy(M.data(), hm, M.size() * 4);
  // row s of M = what rank s sends to each owner
  std::vector<int64_t> soff((size_t)W + 1, 0), roff((size_t)W + 1, 0);
  for (int p = 0; p < W; p++) {
    soff[(size_t)p + 1] = soff[(size_t)p] + M[(size_t)me * W + p];
    roff[(size_t)p + 1] = roff[(size_t)p] + M[(size_t)p * W + me];
  }
  const int64_t nsend = soff[(size_t)W], nrecv = roff[(size_t)W];
  std::vector<uint32_t> cur((size_t)W);
  for (int p = 0; p < W; p++) cur[(size_t)p] = (uint32_t)soff[(size_t)p];
  uint32_t* d_cur = arena_alloc<uint32_t>(ctx, W);
  HostMsg* d_send = arena_alloc<HostMsg>(ctx, nsend);
  uint64_t* d_sslot = arena_alloc<uint64_t>(ctx, nsend);
  HostMsg* d_recv = arena_alloc<HostMsg>(ctx, nrecv);
  uint32_t* d_reply = arena_alloc<uint32_t>(ctx, nrecv);
  uint32_t* d_back = arena_alloc<uint32_t>(ctx, nsend);
  uint64_t ocap = 1;
  while (ocap < (uint64_t)(2 * std::max<int64_t>(nrecv, 1))) ocap <<= 1;
  uint64_t* d_okeys = arena_alloc<uint64_t>(ctx, (int64_t)ocap);
  uint32_t* d_ovals = arena_alloc<uint32_t>(ctx, (int64_t)ocap);
  if (!d_cur || !d_send || !d_sslot || !d_recv || !d_reply || !d_back || !d_okeys || !d_ovals)
    return ctx->fail(YRWI_E_NOMEM, "arena");
  if (upload(ctx, d_cur, cur)) return YRWI_E_HIP;
  HIPCHK(ctx, hipMemsetAsync(d_okeys, 0, ocap * 8, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync(d_ovals, 0, ocap * 4, ctx->stream));
  if (launch_host_pack(d_hkeys, d_hcnt, d_sb, nq, nslots, W, d_cur, d_send, d_sslot, ctx->stream, hkey))
    return ctx->fail(YRWI_E_HIP, "host pack");
  {
    std::vector<Xfer> snd, rcv;
    for (int p = 0; p < W; p++) {
      snd.push_back({p, d_send + soff[(size_t)p], (size_t)(soff[(size_t)p + 1] - soff[(size_t)p]) * sizeof(HostMsg)});
      rcv.push_back({p, d_recv + roff[(size_t)p], (size_t)(roff[(size_t)p + 1] - roff[(size_t)p]) * sizeof(HostMsg)});
    }
    if (int rc = coll_exchange(ctx, snd, rcv)) return rc;
  }
  if (launch_host_owner(d_recv, nrecv, d_okeys, d_ovals, ocap - 1, d_gmax, d_reply, ctx->stream))
    return ctx->fail(YRWI_E_HIP, "host owner");
  if (int rc = coll_allreduce_i32(ctx, d_gmax, (size_t)nq, true)) return rc;
  {
    std::vector<Xfer> snd, rcv;  // replies to what p sent me; totals for what I sent p
    for (int p = 0; p < W; p++) {
      snd.push_back({p, d_reply + roff[(size_t)p], (size_t)(roff[(size_t)p + 1] - roff[(size_t)p]) * 4});
      rcv.push_back({p, d_back + soff[(size_t)p], (size_t)(soff[(size_t)p + 1] - soff[(size_t)p]) * 4});
    }
    if (int rc = coll_exchange(ctx, snd, rcv)) return rc;
  }
  if (launch_host_apply(d_back, d_sslot, nsend, d_hcnt, d_ss, d_gmax, nq, ctx->stream))
    return ctx->fail(YRWI_E_HIP, "host apply");
  return 0;
}

// Normalise (+ cross-shard exchange), then either score+top-k (hits) or all scores.
static int run_rank_phase(Lane* ctx, std::vector<Plan>& plans, int32_t kmax, yrwi_hit* h_hits,
                          int32_t* h_nout, int64_t* h_scores_all, yrwi_stats* st, Timing* tm, bool exchange = true) {
  const int nq = (int)plans.size();
  const int W = exchange ? ctx->world : 1;
  const bool shx = exchange && ctx->sharded;  // the url-hash-shard protocol
  std::vector<RankQ> rq((size_t)nq);
  std::vector<int64_t> chunk_base((size_t)nq), slot_base((size_t)nq + 1);
  int64_t chunks = 0, nslots = 0;
  bool any_auth = false;
  for (int qi = 0; qi < nq; qi++) {
    Plan& P = plans[(size_t)qi];
    RankQ& R = rq[(size_t)qi];
    std::memset(&R, 0, sizeof(R));
    R.feat = P.cont.feat;
    R.uid = P.cont.uid;
    R.ekhi = P.cont.uid ? nullptr : P.cont.khi;
    R.eklo = P.cont.uid ? nullptr : P.cont.klo;
    R.dkhi = ctx->dkhi;
    R.dklo = ctx->dklo;
    R.removed = P.removed;
    R.n = P.empty ? 0 : P.cont.n;
    R.pieces = P.empty || P.removed ? nullptr : P.pieces;
    R.npieces = R.pieces ? P.npieces : 0;
    R.ngroups = ceil_div(R.npieces, 64);
    R.nchunks = ceil_div(R.n, CHUNK);
    R.chunk_base = chunks;
    chunk_base[(size_t)qi] = chunks;
    chunks += R.nchunks;
    R.prof = P.prof;
    R.lang[0] = P.lang[0];
    R.lang[1] = P.lang[1];
    R.lang_ok = P.lang_ok;
    R.now_ms = P.now_ms;
    R.k = P.k;
    R.want_authority = P.prof.coeff_authority > 12 && R.n > 0;
    R.idx_tag = shx ? (uint32_t)ctx->rank << 28 : 0u;
    R.doubledom = P.filter && P.filter->skip_double_dom ? 1 : 0;
    R.host_rec = ctx->host_ids && P.cont.uid != nullptr ? 1 : 0;  // index records: dense host ids
    R.kout = P.k;
    if (R.doubledom) R.k = YRWI_MAX_K;  // pullOneRWI draws from the whole rwiStack (max_results_rwi)
    // identical on every rank (same queries): decides the collective host-count exchange
    if (P.prof.coeff_authority > 12) any_auth = true;
    if (R.want_authority) {
      uint64_t cap = 1;
      while (cap < (uint64_t)(2 * R.n)) cap <<= 1;
      R.hmask = cap - 1;
      slot_base[(size_t)qi] = nslots;
      nslots += (int64_t)cap;
    } else {
      slot_base[(size_t)qi] = nslots;
    }
    if (st) {
      st->joined += R.n;
      st->bytes_alg += 23 * (int64_t)P.seq.size() * R.n;  // ranking feature bytes per surviving posting and term
      st->bytes_features += 23 * (int64_t)P.seq.size() * R.n;
      st->bytes_alg_capped += 23 * (int64_t)P.seq.size() * R.n;
    }
  }
  slot_base[(size_t)nq] = nslots;
  // authority host tables of all queries, one allocation
  uint64_t* d_hkeys = nullptr;
  uint32_t* d_hcnt = nullptr;
  if (nslots > 0) {
    d_hkeys = arena_alloc<uint64_t>(ctx, nslots);
    d_hcnt = arena_alloc<uint32_t>(ctx, nslots);
    if (!d_hkeys || !d_hcnt) return ctx->fail(YRWI_E_NOMEM, "arena");
    HIPCHK(ctx, hipMemsetAsync(d_hkeys, 0, (size_t)nslots * 8, ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(d_hcnt, 0, (size_t)nslots * 4, ctx->stream));
    for (int qi = 0; qi < nq; qi++) {
      RankQ& R = rq[(size_t)qi];
      if (!R.want_authority) continue;
      R.hkeys = d_hkeys + slot_base[(size_t)qi];
      R.hcnt = d_hcnt + slot_base[(size_t)qi];
    }
  }
  // authority by partition (RankQ::ecnt; one context, records with host ids): each
  // query's hosts hashed into ~HPART_TARGET-element buckets, per-element counts
  int64_t hp_hist = 0, hp_elems = 0, hp_buckets = 0;
  std::vector<int2> bq;
  const char* hpm = getenv("YRWI_HPART_MAXB");  // (tests: fewer buckets, so large queries overflow the LDS tables)
  const int64_t maxb = hpm ? std::max(1, std::min(HPART_MAXS, atoi(hpm))) : HPART_MAXS;
  for (int qi = 0; qi < nq; qi++) {
    RankQ& R = rq[(size_t)qi];
    if (!R.want_authority || !R.host_rec || shx) continue;
    R.hp_nb = (int32_t)std::min<int64_t>(maxb, std::max<int64_t>(1, ceil_div(R.n, HPART_TARGET)));
    R.hp_hoff = hp_hist;
    hp_hist += R.nchunks * R.hp_nb;
    for (int32_t s = 0; s < R.hp_nb; s++) bq.push_back(make_int2(qi, s));
    hp_buckets += R.hp_nb;
  }
  int32_t *d_hist = nullptr, *d_hoffs = nullptr, *d_ecnt = nullptr;
  uint2* d_part = nullptr;
  int2* d_bq = nullptr;
  void* d_hptmp = nullptr;
  size_t hp_tmp = 0;
  if (hp_buckets > 0) {
    for (int qi = 0; qi < nq; qi++) if (rq[(size_t)qi].hp_nb) hp_elems += rq[(size_t)qi].n;
    hp_tmp = host_part_tmp_bytes(hp_hist);
    d_hist = arena_alloc<int32_t>(ctx, hp_hist + 1);
    d_hoffs = arena_alloc<int32_t>(ctx, hp_hist + 1);
    d_ecnt = arena_alloc<int32_t>(ctx, hp_elems);
    d_part = arena_alloc<uint2>(ctx, hp_elems);
    d_bq = arena_alloc<int2>(ctx, hp_buckets);
    d_hptmp = arena_alloc<uint8_t>(ctx, (int64_t)std::max<size_t>(hp_tmp, 1));
    if (!d_hist || !d_hoffs || !d_ecnt || !d_part || !d_bq || !d_hptmp) return ctx->fail(YRWI_E_NOMEM, "arena");
    HIPCHK(ctx, hipMemsetAsync(d_hist + hp_hist, 0, 4, ctx->stream));  // the scan's extra entry: the total
    int64_t eb = 0;
    for (int qi = 0; qi < nq; qi++) {
      RankQ& R = rq[(size_t)qi];
      if (!R.hp_nb) continue;
      R.ecnt = d_ecnt + eb;
      R.hp_hist = d_hist;
      eb += R.n;
    }
    if (upload(ctx, d_bq, bq)) return YRWI_E_HIP;
  }
  // addRWIs constraints: one FilterQ per filtered query, key arrays and flag counters
  std::vector<int> fidx((size_t)nq, -1);
  int nf = 0;
  bool any_dd = false, any_flagcount = false;
  for (int qi = 0; qi < nq; qi++) {
    if (plans[(size_t)qi].filter) fidx[(size_t)qi] = nf++;
    if (rq[(size_t)qi].doubledom) any_dd = true;
    if (plans[(size_t)qi].filter && plans[(size_t)qi].filter->flagcount) any_flagcount = true;
  }
  int32_t* d_flag = nullptr;
  if (nf > 0) {
    std::vector<FilterQ> fq((size_t)nf);
    std::vector<uint64_t> sx, uh;
    std::vector<uint8_t> ul;
    std::vector<int64_t> sx0((size_t)nf), uh0((size_t)nf);
    for (int qi = 0; qi < nq; qi++) {
      if (fidx[(size_t)qi] < 0) continue;
      const yrwi_filter& F = *plans[(size_t)qi].filter;
      FilterQ& G = fq[(size_t)fidx[(size_t)qi]];
      std::vector<uint64_t> v;
      std::vector<KeyT> u;
      build_filterq(F, &G, &v, &u);
      sx0[(size_t)fidx[(size_t)qi]] = (int64_t)sx.size();
      sx.insert(sx.end(), v.begin(), v.end());
      uh0[(size_t)fidx[(size_t)qi]] = (int64_t)uh.size();
      for (auto& k : u) { uh.push_back(k.hi); ul.push_back((uint8_t)k.lo); }
    }
    FilterQ* d_fq = arena_alloc<FilterQ>(ctx, nf);
    uint64_t* d_sx = arena_alloc<uint64_t>(ctx, (int64_t)sx.size());
    uint64_t* d_uh = arena_alloc<uint64_t>(ctx, (int64_t)uh.size());
    uint8_t* d_ul = arena_alloc<uint8_t>(ctx, (int64_t)ul.size());
    d_flag = any_flagcount ? arena_alloc<int32_t>(ctx, (int64_t)nf * 32) : nullptr;
    if (!d_fq || !d_sx || !d_uh || !d_ul || (any_flagcount && !d_flag)) return ctx->fail(YRWI_E_NOMEM, "arena");
    if (d_flag) HIPCHK(ctx, hipMemsetAsync(d_flag, 0, (size_t)nf * 32 * 4, ctx->stream));
    for (int qi = 0; qi < nq; qi++) {
      const int f = fidx[(size_t)qi];
      if (f < 0) continue;
      FilterQ& G = fq[(size_t)f];
      G.siteex = d_sx + sx0[(size_t)f];
      G.url_hi = d_uh + uh0[(size_t)f];
      G.url_lo = d_ul + uh0[(size_t)f];
      G.flagcount = plans[(size_t)qi].filter->flagcount ? d_flag + (int64_t)f * 32 : nullptr;
      rq[(size_t)qi].filt = d_fq + f;
    }
    if (upload(ctx, d_fq, fq, d_sx, sx, d_uh, uh, d_ul, ul))
      return YRWI_E_HIP;
  }
  // flag counters back to the callers' filters (summed over the shards)
  auto flagcounts_out = [&]() -> int {
    if (!d_flag) return 0;
    if (shx)
      if (int rc = coll_allreduce_i32(ctx, d_flag, (size_t)nf * 32, false)) return rc;
    const uint8_t* hf = readback(ctx, &ctx->down_stage, d_flag, (int64_t)nf * 32, 4, 4);
    if (!hf) return YRWI_E_HIP;
    HIPCHK(ctx, lane_sync(ctx));
    std::vector<int32_t> h((size_t)nf * 32);
    std::memcpy(h.data(), hf, h.size() * 4);
    for (int qi = 0; qi < nq; qi++)
      if (fidx[(size_t)qi] >= 0 && plans[(size_t)qi].filter->flagcount)
        std::memcpy(plans[(size_t)qi].filter->flagcount, &h[(size_t)fidx[(size_t)qi] * 32], 32 * 4);
    return 0;
  };
  RankQ* d_q = arena_alloc<RankQ>(ctx, nq);
  int64_t* d_cb = arena_alloc<int64_t>(ctx, nq);
  ChunkSum* d_cs = arena_alloc<ChunkSum>(ctx, chunks);
  ShardSum* d_ss = arena_alloc<ShardSum>(ctx, nq);
  ShardSum* d_all = shx ? arena_alloc<ShardSum>(ctx, (int64_t)nq * W) : d_ss;
  NormState* d_norm = arena_alloc<NormState>(ctx, nq);
  if (!d_q || !d_cb || !d_cs || !d_ss || !d_all || !d_norm) return ctx->fail(YRWI_E_NOMEM, "arena");
  std::vector<int32_t> chunk_q((size_t)chunks);
  for (int qi = 0; qi < nq; qi++)
    for (int64_t c = 0; c < rq[(size_t)qi].nchunks; c++) chunk_q[(size_t)(chunk_base[(size_t)qi] + c)] = qi;
  int32_t* d_cq = arena_alloc<int32_t>(ctx, chunks);
  if (!d_cq) return ctx->fail(YRWI_E_NOMEM, "arena");
  // groups of the compaction's pieces (k_piece_merge): (query, group) of each
  std::vector<int2> group_q;
  for (int qi = 0; qi < nq; qi++)
    for (int64_t g = 0; g < rq[(size_t)qi].ngroups; g++) group_q.push_back(make_int2(qi, (int32_t)g));
  int2* d_gq = nullptr;
  if (!group_q.empty()) {
    ChunkSum* d_groups = arena_alloc<ChunkSum>(ctx, (int64_t)group_q.size());
    d_gq = arena_alloc<int2>(ctx, (int64_t)group_q.size());
    if (!d_groups || !d_gq) return ctx->fail(YRWI_E_NOMEM, "arena");
    int64_t gb = 0;
    for (int qi = 0; qi < nq; qi++) {
      RankQ& R = rq[(size_t)qi];
      R.groups = R.ngroups ? d_groups + gb : nullptr;
      gb += R.ngroups;
    }
    if (upload(ctx, d_gq, group_q)) return YRWI_E_HIP;
  }
  if (upload(ctx, d_q, rq, d_cb, chunk_base, d_cq, chunk_q)) return YRWI_E_HIP;
  HIPCHK(ctx, hipMemsetAsync(d_ss, 0, sizeof(ShardSum) * nq, ctx->stream));
  hipEvent_t sp = span_open(ctx, tm);
  hipEvent_t rmid = tm ? ctx->event() : nullptr;  // after k_reduce, before k_shard_fin
  bool reduce = false;  // a query without the compaction's pieces
  for (int qi = 0; qi < nq; qi++) reduce |= !rq[(size_t)qi].pieces && rq[(size_t)qi].nchunks > 0;
  if (launch_reduce(d_q, d_cb, d_cq, nq, chunks, d_cs, d_ss, ctx->stream, rmid, hp_buckets > 0, reduce, d_gq,
                    (int64_t)group_q.size()))
    return ctx->fail(YRWI_E_HIP, "reduce launch");
  if (hp_buckets > 0 &&
      launch_host_part(d_q, d_cq, chunks, d_hist, d_hoffs, hp_hist, d_hptmp, hp_tmp, d_part, d_bq,
                       (int32_t)hp_buckets, d_ss, ctx->stream))
    return ctx->fail(YRWI_E_HIP, "host count launch");
  span_close(ctx, tm, sp);
  if (tm) tm->kreduce.push_back({sp, rmid});  // k_reduce alone: the population rocprofv3 averages
  if (st) {
    st->n_rank_passes++;
    for (int qi = 0; qi < nq; qi++) {
      const int64_t n = rq[(size_t)qi].n;
      if (!rq[(size_t)qi].pieces) st->bytes_reduce += (int64_t)FEAT_BYTES * n + (rq[(size_t)qi].removed ? n : 0);
      st->bytes_score += (int64_t)FEAT_BYTES * n + (rq[(size_t)qi].removed ? n : 0);
    }
  }
  if (shx && any_auth) {
    int rc2 = exchange_host_counts(ctx, nq, nslots, slot_base, d_hkeys, d_hcnt, d_ss);
    if (rc2) return rc2;
  }
  if (shx) {
    if (int rc = coll_allgather(ctx, d_ss, d_all, sizeof(ShardSum) * nq)) return rc;
  }
  sp = span_open(ctx, tm);
  if (launch_combine(d_q, nq, d_all, W, d_norm, ctx->stream)) return ctx->fail(YRWI_E_HIP, "combine launch");
  span_close(ctx, tm, sp);
  if (tm) { tm->tn = ctx->event(); hipEventRecord(tm->tn, ctx->stream); }

  if (h_scores_all) {  // yrwi_normalize_score
    int64_t* d_sc = arena_alloc<int64_t>(ctx, rq[0].n);
    if (!d_sc) return ctx->fail(YRWI_E_NOMEM, "arena");
    if (launch_score_all(d_q, d_cq, nq, chunks, d_norm, d_sc, ctx->stream)) return ctx->fail(YRWI_E_HIP, "score launch");
    HIPCHK(ctx, hipMemcpyAsync(h_scores_all, d_sc, sizeof(int64_t) * rq[0].n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, lane_sync(ctx));
    NormState nsh;
    HIPCHK(ctx, hipMemcpy(&nsh, d_norm, sizeof(nsh), hipMemcpyDeviceToHost));
    if (nsh.D < 0) return ctx->fail(YRWI_E_UNSUPPORTED, "distance fold summary overflow");
    return 0;
  }

  // ---- score + per-chunk top-k
  int32_t keff = 1;
  for (auto& R : rq) keff = std::max(keff, R.k);
  const int32_t kc = std::min<int32_t>(keff, CHUNK);  // per-chunk candidate list stride
  Cand* d_cand = arena_alloc<Cand>(ctx, std::max<int64_t>(chunks, 1) * kc);
  int32_t* d_ccnt = arena_alloc<int32_t>(ctx, std::max<int64_t>(chunks, 1));
  if (!d_cand || !d_ccnt) return ctx->fail(YRWI_E_NOMEM, "arena");
  // d_zero[0]: a zero count (queries without chunks); d_zero[1]: k_score's redo count
  int32_t* d_zero = arena_alloc<int32_t>(ctx, 2);
  int32_t* d_redo = arena_alloc<int32_t>(ctx, std::max<int64_t>(chunks, 1));
  if (!d_zero || !d_redo) return ctx->fail(YRWI_E_NOMEM, "arena");
  HIPCHK(ctx, hipMemsetAsync(d_zero, 0, 2 * sizeof(int32_t), ctx->stream));
  sp = span_open(ctx, tm);
  // chunk order for k_score: every query's chunk 0, then every chunk 1, ... so that
  // a big query's later chunks run after its threshold is set (PruneP)
  std::vector<int32_t> order((size_t)chunks * 2);  // (chunk, query) pairs
  {
    // counting sort by chunk index c (stable in query order): O(chunks + max chunks)
    int64_t maxc = 0;
    for (auto& R : rq) maxc = std::max(maxc, R.nchunks);
    std::vector<int64_t> at((size_t)maxc + 1, 0);
    for (auto& R : rq)
      for (int64_t c = 0; c < R.nchunks; c++) at[(size_t)c + 1]++;
    for (int64_t c = 0; c < maxc; c++) at[(size_t)c + 1] += at[(size_t)c];
    for (int qi = 0; qi < nq; qi++)
      for (int64_t c = 0; c < rq[(size_t)qi].nchunks; c++) {
        const size_t o = (size_t)at[(size_t)c]++;
        order[2 * o] = (int32_t)(chunk_base[(size_t)qi] + c);
        order[2 * o + 1] = qi;
      }
  }
  int32_t* d_order = arena_alloc<int32_t>(ctx, 2 * chunks);
  unsigned long long* d_tq = arena_alloc<unsigned long long>(ctx, nq);
  uint8_t* d_qtab = arena_alloc<uint8_t>(ctx, (int64_t)nq * (int64_t)score_qtab_bytes());
  if (!d_order || !d_tq || !d_qtab) return ctx->fail(YRWI_E_NOMEM, "arena");
  if (upload(ctx, d_order, order)) return YRWI_E_HIP;
  HIPCHK(ctx, hipMemsetAsync(d_tq, 0, sizeof(unsigned long long) * (size_t)nq, ctx->stream));
  // (a separate launch of every query's first chunk, so that all later chunks
  // start with a threshold, measured 39 + 86 us against 99 us for one launch:
  // the seed launch is one round of full-length blocks)
  const int64_t seed = 0;
  // the k_score launches alone (the population rocprofv3 averages): from right
  // before them to before k_score_full
  hipEvent_t s0 = span_open(ctx, tm);
  hipEvent_t smid = tm ? ctx->event() : nullptr;
  if (launch_score(d_q, d_cq, d_order, nq, chunks, seed, d_norm, d_cand, d_ccnt, kc, d_redo, d_zero + 1, d_tq,
                   d_qtab, ctx->stream, smid))
    return ctx->fail(YRWI_E_HIP, "score launch");
  span_close(ctx, tm, sp);
  if (tm) tm->kscore.push_back({s0, smid});
  // ---- top-k passes over groups of candidate lists until one list per query;
  // a query with a single list (one chunk) is final as it stands
  std::vector<const Cand*> fptr((size_t)nq);
  std::vector<const int32_t*> fcnt((size_t)nq);
  std::vector<int64_t> lists((size_t)nq), lbase((size_t)nq);
  for (int qi = 0; qi < nq; qi++) {
    lists[(size_t)qi] = rq[(size_t)qi].nchunks;
    lbase[(size_t)qi] = chunk_base[(size_t)qi];
    fptr[(size_t)qi] = d_cand + chunk_base[(size_t)qi] * kc;
    fcnt[(size_t)qi] = lists[(size_t)qi] ? d_ccnt + chunk_base[(size_t)qi] : d_zero;
  }
  const Cand* cur = d_cand;
  const int32_t* curc = d_ccnt;
  int32_t in_stride = kc;
  while (true) {
    const int64_t G = std::max<int64_t>(2, std::min<int64_t>(64, topq_capacity(keff) / in_stride));
    std::vector<int64_t> gb;
    std::vector<int32_t> gn, gk;
    std::vector<int> part;
    for (int qi = 0; qi < nq; qi++) {
      const int64_t L = lists[(size_t)qi];
      if (L <= 1) continue;
      const int64_t ng = ceil_div(L, G);
      const int64_t first = (int64_t)gb.size();
      for (int64_t g = 0; g < ng; g++) {
        gb.push_back(lbase[(size_t)qi] + g * G);
        gn.push_back((int32_t)std::min<int64_t>(G, L - g * G));
        gk.push_back(rq[(size_t)qi].k);
      }
      lists[(size_t)qi] = ng;
      lbase[(size_t)qi] = first;
      part.push_back(qi);
    }
    if (gb.empty()) break;
    const int64_t ngr = (int64_t)gb.size();
    int64_t* d_gb = arena_alloc<int64_t>(ctx, ngr);
    int32_t* d_gn = arena_alloc<int32_t>(ctx, ngr);
    int32_t* d_gk = arena_alloc<int32_t>(ctx, ngr);
    Cand* d_out = arena_alloc<Cand>(ctx, ngr * keff);
    int32_t* d_oc = arena_alloc<int32_t>(ctx, ngr);
    if (!d_gb || !d_gn || !d_gk || !d_out || !d_oc) return ctx->fail(YRWI_E_NOMEM, "arena");
    if (upload(ctx, d_gb, gb, d_gn, gn, d_gk, gk)) return YRWI_E_HIP;
    hipEvent_t sq = span_open(ctx, tm);
    if (launch_topq(d_gb, d_gn, d_gk, ngr, cur, curc, in_stride, keff, d_out, d_oc, ctx->stream))
      return ctx->fail(YRWI_E_HIP, "top-k launch");
    span_close(ctx, tm, sq);
    for (int qi : part) {
      fptr[(size_t)qi] = d_out + lbase[(size_t)qi] * keff;
      fcnt[(size_t)qi] = d_oc + lbase[(size_t)qi];
    }
    in_stride = keff;
    cur = d_out;
    curc = d_oc;
  }
  const Cand** d_fptr = arena_alloc<const Cand*>(ctx, nq);
  const int32_t** d_fcnt = arena_alloc<const int32_t*>(ctx, nq);
  // Results go straight into pinned host memory -- the caller's buffer when it
  // came from yrwi_host_alloc, else this lane's landing buffer (then copied out
  // per query).  One GPU: k_emit writes them (doubledom queries: their stacks,
  // ordered by k_pull).  Sharded: every shard's stack is gathered, merged on the
  // device (k_gmerge_*) and pulled (k_pull); every rank ends with the same lists.
  const int32_t kint = any_dd ? YRWI_MAX_K : kmax;  // stack stride
  const size_t hb = sizeof(yrwi_hit) * (size_t)nq * kmax, hb_al = (hb + 255) & ~(size_t)255;
  const size_t nb = sizeof(int32_t) * (size_t)nq;
  yrwi_hit* d_hits = nullptr;
  int32_t* d_nout = nullptr;
  const bool direct = ctx->hostreg && ctx->hostreg->contains(h_hits, hb) && ctx->hostreg->contains(h_nout, nb);
  uint8_t* land = nullptr;
  {
    void* hp = h_hits;
    void* np = h_nout;
    if (!direct) {
      land = stage_reserve(ctx, &ctx->out_stage, hb_al + nb, true);
      if (!land) return YRWI_E_HIP;
      hp = land;
      np = land + hb_al;
    }
    // the emit kernels write the pinned destination directly (a DMA copy from a
    // device buffer instead measured 1.17 vs 1.07 ms per C2 step)
    HIPCHK(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&d_hits), hp, 0));
    HIPCHK(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&d_nout), np, 0));
  }
  if (!d_fptr || !d_fcnt) return ctx->fail(YRWI_E_NOMEM, "arena");
  if (upload(ctx, d_fptr, fptr, d_fcnt, fcnt)) return YRWI_E_HIP;
  std::vector<int32_t> hD;  // max-distance fold state per query (overflow check)
  const uint8_t* hD_land = nullptr;
  if (!shx) {
    sp = span_open(ctx, tm);
    if (launch_emit(d_q, nq, d_fptr, d_fcnt, kmax, d_hits, d_nout, 0, ctx->stream))
      return ctx->fail(YRWI_E_HIP, "emit launch");
    span_close(ctx, tm, sp);
    if (any_dd) {
      yrwi_hit* d_stack = arena_alloc<yrwi_hit>(ctx, (int64_t)nq * kint);
      int32_t* d_scnt = arena_alloc<int32_t>(ctx, nq);
      if (!d_stack || !d_scnt) return ctx->fail(YRWI_E_NOMEM, "arena");
      sp = span_open(ctx, tm);
      if (launch_emit(d_q, nq, d_fptr, d_fcnt, kint, d_stack, d_scnt, 2, ctx->stream) ||
          launch_pull(d_q, nq, d_stack, d_scnt, kint, 1, kmax, d_hits, d_nout, ctx->stream))
        return ctx->fail(YRWI_E_HIP, "doubledom launch");
      span_close(ctx, tm, sp);
    }
  } else {
    yrwi_hit* d_mine = arena_alloc<yrwi_hit>(ctx, (int64_t)nq * kint);
    int32_t* d_mcnt = arena_alloc<int32_t>(ctx, nq);
    yrwi_hit* d_allh = arena_alloc<yrwi_hit>(ctx, (int64_t)nq * kint * W);
    int32_t* d_alln = arena_alloc<int32_t>(ctx, (int64_t)nq * W);
    uint32_t* d_slot = arena_alloc<uint32_t>(ctx, (int64_t)nq * kint * W);
    uint8_t* d_dup = arena_alloc<uint8_t>(ctx, (int64_t)nq * kint * W);
    yrwi_hit* d_stack = arena_alloc<yrwi_hit>(ctx, (int64_t)nq * kint);
    int32_t* d_scnt = arena_alloc<int32_t>(ctx, nq);
    if (!d_mine || !d_mcnt || !d_allh || !d_alln || !d_slot || !d_dup || !d_stack || !d_scnt)
      return ctx->fail(YRWI_E_NOMEM, "arena");
    sp = span_open(ctx, tm);
    if (launch_emit(d_q, nq, d_fptr, d_fcnt, kint, d_mine, d_mcnt, 1, ctx->stream))
      return ctx->fail(YRWI_E_HIP, "emit launch");
    span_close(ctx, tm, sp);
    if (int rc = coll_allgather(ctx, d_mine, d_allh, sizeof(yrwi_hit) * (size_t)nq * kint)) return rc;
    if (int rc = coll_allgather(ctx, d_mcnt, d_alln, sizeof(int32_t) * (size_t)nq)) return rc;
    if (ctx->release_after_final) turn_release(ctx);  // the next batch part's collectives may follow now
    sp = span_open(ctx, tm);
    if (launch_gmerge(d_q, d_allh, d_alln, W, nq, kint, d_slot, d_dup, d_stack, d_scnt, ctx->stream) ||
        launch_pull(d_q, nq, d_stack, d_scnt, kint, 0, kmax, d_hits, d_nout, ctx->stream))
      return ctx->fail(YRWI_E_HIP, "shard merge launch");
    span_close(ctx, tm, sp);
    hD_land = readback(ctx, &ctx->down_stage, reinterpret_cast<const uint8_t*>(d_norm) + offsetof(NormState, D), nq,
                       4, (int64_t)sizeof(NormState));
    if (!hD_land) return YRWI_E_HIP;
  }
  if (tm) { tm->ts = ctx->event(); hipEventRecord(tm->ts, ctx->stream); }
  HIPCHK(ctx, lane_sync(ctx));
  if (hD_land) {
    hD.resize((size_t)nq);
    std::memcpy(hD.data(), hD_land, (size_t)nq * 4);
  }
  for (int32_t D : hD)
    if (D < 0) return ctx->fail(YRWI_E_UNSUPPORTED, "distance fold summary overflow");
  if (!direct) {
    std::memcpy(h_nout, land + hb_al, nb);
    for (int qi = 0; qi < nq; qi++)
      std::memcpy(h_hits + (size_t)qi * kmax, land + sizeof(yrwi_hit) * (size_t)qi * kmax,
                  sizeof(yrwi_hit) * (size_t)std::max(0, std::min(h_nout[qi], kmax)));
  }
  return flagcounts_out();
}

static int64_t now_ns() {
  return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Plan and run queries q[0, nq) on lane L; results at out (row stride kmax).
// Every field of *st is this part's own (the caller sums parts).
// Upper bound of the arena bytes one query takes in a pass: per fold step the
// join's tile descriptors (~1 B per 64 input postings), its matched pairs (12 B
// each, at most the smaller side) and the joined container (url id + 32-byte
// record: 36 B per row, at most the smallest list), then the rank phase over
// that container (exclusion marks, chunk summaries, candidates: ~48 B per row).
// Scratch bytes a query is expected to take in a pass: 48 B per slot of its
// smallest list and fold step (a step-by-step container at its bound min(nA, nB);
// a chained fold's pair slots, later-list rows, tile arrays and output), plus the
// ranked container.  (A tighter estimate for chained folds -- pairs and rows
// once, the output from the lists' densities -- put C4's eight lanes past the
// device's memory as their outputs grew the arenas: profiles/archive/r04_c4_host.txt.)
static int64_t scratch_estimate(const Plan& P) {
  if (P.empty || P.seq.empty()) return 4096;
  int64_t sum = 0, nmin = INT64_MAX;
  for (const ListRec* l : P.seq) {
    sum += l->n;
    nmin = std::min(nmin, l->n);
  }
  for (const ListRec* l : P.excl) sum += l->n;
  return sum / 64 + (48 * (int64_t)(P.seq.size() - 1) + 48) * nmin + 65536;
}

// Scratch budget of one pass (YRWI_SCRATCH_GB per lane, default 192 GiB / lanes).  A
// batch whose queries need more runs as consecutive passes over query ranges;
// sharded contexts never split (every rank must issue the same collectives, and
// the estimate depends on the local shard), so they keep one pass per batch.
static int64_t scratch_budget(const Lane* L) {
  if (L->sharded) return INT64_MAX;
  // per lane: YRWI_SCRATCH_GB, else the device memory left beside the resident
  // index (measured after it was built, ensure_url_ids: free memory + the lanes'
  // arenas then - 8 GiB headroom) shared by the lanes, at most 192 GiB in all (C4:
  // 16 GiB per lane ran 7 passes a batch at 10.3 ms/step, 24 GiB 9.86, 32 GiB 9.73
  // -- the passes' fixed kernels and syncs; profiles/archive/r04_scratch_c4.txt)
  const char* e = getenv("YRWI_SCRATCH_GB");
  if (e) return (int64_t)(std::max(atof(e), 0.001) * (double)(1ll << 30));
  const int64_t cap = (int64_t)192 << 30;
  const int64_t tot = L->scratch_total ? L->scratch_total->load() : 0;
  const int64_t all = tot > 0 ? std::min(tot, cap) : cap;
  return std::max<int64_t>(all / std::max(1, L->nlanes), (int64_t)256 << 20);
}

// the scratch budget's base (scratch_budget): device memory free beside the index,
// dictionary and bitmaps, plus what the lanes' arenas hold now, minus headroom
void yrwi::measure_scratch(CtxBase* ctx) {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  int64_t arenas = 0;
  for (Lane* L : ctx->lanes) arenas += (int64_t)L->arena.capacity();
  ctx->scratch_total = std::max<int64_t>((int64_t)fr + arenas - ((int64_t)8 << 30), (int64_t)1 << 30);
}

static int run_batch_part_(const yrwi_ctx* ix, Lane* L, const yrwi_query_desc* q, int32_t nq, int32_t kmax,
                           yrwi_hit* out, int32_t* nout, yrwi_stats* st);

static int run_batch_part(const yrwi_ctx* ix, Lane* L, const yrwi_query_desc* q, int32_t nq, int32_t kmax,
                          yrwi_hit* out, int32_t* nout, yrwi_stats* st) {
  L->enter();
  const int64_t seq = L->seq;  // (passing the turn after the final collective clears L->seq)
  const int rc = run_batch_part_(ix, L, q, nq, kmax, out, nout, st);
  // peers waiting on this part's exchanges fail fast; later parts are unaffected
  if (rc && L->hostx) hostx_abort(L->hostx, seq);
  turn_release(L);  // error paths, parts without collectives: the turn still passes in order
  L->release_after_final = false;
  L->leave();
  return rc;
}

static int run_batch_part_(const yrwi_ctx* ix, Lane* L, const yrwi_query_desc* q, int32_t nq, int32_t kmax,
                           yrwi_hit* out, int32_t* nout, yrwi_stats* st) {
  const int64_t t0 = now_ns();
  const int64_t r0 = t_realloc;
  int64_t tp = 0, tj = 0, tr = 0, w0 = L->wait_ns, wj = 0;
  std::vector<Plan> all((size_t)nq);
  for (int i = 0; i < nq; i++) {
    int rc = plan_query(ix, L, q[i], &all[(size_t)i]);
    if (rc) return rc;
    if (st) st->postings_in += all[(size_t)i].postings_in;
  }
  // url selections: restricted list sizes first (J1/J2/J3 decide on them)
  if (int rc = resolve_selections(L, all)) return rc;
  // J1/J2 on global list sizes (one exchange of the batch's term sizes when sharded,
  // through this lane's arena and staging)
  if (L->sharded && begin_pass(L)) return YRWI_E_HIP;
  if (int rc = plan_batch(L, all)) return rc;
  tp = now_ns() - t0;
  const int64_t budget = scratch_budget(L);
  int npass = 0;
  for (int g0 = 0; g0 < nq;) {
    npass++;
    int g1 = g0;
    int64_t need = 0;
    while (g1 < nq) {
      const int64_t e = scratch_estimate(all[(size_t)g1]);
      if (g1 > g0 && need + e > budget) break;
      need += e;
      g1++;
    }
    std::vector<Plan> plans(std::make_move_iterator(all.begin() + g0), std::make_move_iterator(all.begin() + g1));
    L->release_after_final = g1 >= nq;
    if (begin_pass(L)) return YRWI_E_HIP;
    // HIP events (per-kernel timing) only when the caller asked for statistics
    Timing tm;
    Timing* tmp = st ? &tm : nullptr;
    if (tmp) {
      tm.t0 = L->event();
      hipEventRecord(tm.t0, L->stream);
    }
    const int64_t tj0 = now_ns(), wj0 = L->wait_ns;
    int rc = run_join_phase(L, plans, st, tmp);
    if (rc) return rc;
    tj += now_ns() - tj0;
    wj += L->wait_ns - wj0;
    const int64_t tr0 = now_ns();
    if (tmp) {
      tm.tj = L->event();
      hipEventRecord(tm.tj, L->stream);
    }
    rc = run_rank_phase(L, plans, kmax, out + (size_t)g0 * kmax, nout + g0, nullptr, st, tmp);
    if (rc) return rc;
    tr += now_ns() - tr0;
    if (st) {
      if (g1 < nq) HIPCHK(L, lane_sync(L));  // the pass's events must be complete before they are reused
      float ms = 0;
      for (auto& ev : tm.kjoin) {
        if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) st->t_join_ns += (int64_t)(ms * 1e6);
        if (hipEventElapsedTime(&ms, ev[1], ev[2]) == hipSuccess) {
          st->t_probe_ns += (int64_t)(ms * 1e6);
          st->t_probe_all_ns += (int64_t)(ms * 1e6);
        }
      }
      for (auto& ev : tm.kexcl)
        if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) st->t_probe_all_ns += (int64_t)(ms * 1e6);
      for (auto& ev : tm.kcompact)
        if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) st->t_compact_ns += (int64_t)(ms * 1e6);
      for (auto& ev : tm.spans)
        if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) st->t_kernels_ns += (int64_t)(ms * 1e6);
      for (auto& ev : tm.kreduce)
        if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) st->t_reduce_ns += (int64_t)(ms * 1e6);
      for (auto& ev : tm.kscore)
        if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) st->t_scorek_ns += (int64_t)(ms * 1e6);
      for (auto& ev : tm.kchain)
        if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) st->t_chain_ns += (int64_t)(ms * 1e6);
      if (tm.tn && hipEventElapsedTime(&ms, tm.tj, tm.tn) == hipSuccess) st->t_norm_ns += (int64_t)(ms * 1e6);
      if (tm.ts && tm.tn && hipEventElapsedTime(&ms, tm.tn, tm.ts) == hipSuccess) st->t_score_ns += (int64_t)(ms * 1e6);
      // a statistics event that could not be read is not the batch's error: it must
      // not linger as this thread's last HIP error (a later launch check reads it)
      (void)hipGetLastError();
    }
    g0 = g1;
  }
  // An arena that had to grow consolidates now, while this batch's caller still
  // waits for it, not at the start of the lane's next batch (one hipFree +
  // hipMalloc of the whole scratch costs milliseconds).
  if (L->arena.chunks.size() > 1) {
    HIPCHK(L, lane_sync(L));
    L->arena.reset();
    // busy lanes take this size at their next pass (begin_pass)
    size_t h = L->scratch_hint ? L->scratch_hint->load() : 0;
    while (L->scratch_hint && h < L->arena.capacity() &&
           !L->scratch_hint->compare_exchange_weak(h, L->arena.capacity())) {
    }
    // the lanes share one workload: idle lanes take the same size now, so their
    // first batch does not pay for growing (single-lane sharded contexts: none)
    for (Lane* o : ix->lanes)
      if (o != L) o->try_reserve(L->arena.capacity());
  }
  if (st) {
    st->t_total_ns = now_ns() - t0;
    st->n_realloc = (int32_t)(t_realloc - r0);
  }
  return 0;
}

static int check_batch_args(yrwi_ctx* ctx, const yrwi_query_desc* q, int32_t nq, int32_t kmax, yrwi_hit* out,
                            int32_t* nout) {
  if (!ctx || (nq > 0 && (!q || !out || !nout)) || nq < 0 || kmax < 1 || kmax > YRWI_MAX_K) return YRWI_E_ARG;
  return 0;
}

extern "C" int yrwi_settle_scratch(yrwi_ctx* ctx) {
  if (!ctx) return YRWI_E_ARG;
  hipSetDevice(ctx->device);
  drain(ctx);
  size_t a = ctx->scratch_hint.load(), s0 = 0, s1 = 0, s2 = 0;
  for (Lane* L : ctx->lanes) {
    a = std::max(a, L->arena.capacity());
    s0 = std::max(s0, L->stage.cap);
    s1 = std::max(s1, L->out_stage.cap);
    s2 = std::max(s2, L->down_stage.cap);
  }
  for (Lane* L : ctx->lanes) {
    L->arena.reserve(a);  // one chunk of the largest scratch any lane has needed
    if ((s0 && !stage_reserve(L, &L->stage, s0, true)) || (s1 && !stage_reserve(L, &L->out_stage, s1, true)) ||
        (s2 && !stage_reserve(L, &L->down_stage, s2, true)))
      return ctx->take(L, YRWI_E_HIP);
    if (a && L->arena.capacity() < a) return ctx->fail(YRWI_E_NOMEM, "scratch reservation");
  }
  ctx->scratch_hint = a;
  return 0;
}

// wait until no asynchronous batch is in flight (their statuses stay recorded)
void yrwi::drain(CtxBase* ctx) {
  for (Lane* L : ctx->lanes) L->wait();
}

// an authority profile in the batch (ReferenceOrder.cardinal, coeff_authority > 12)
static bool wants_authority(const yrwi_query_desc* q, int32_t nq) {
  for (int32_t i = 0; i < nq; i++)
    if (q[i].profile && q[i].profile->coeff_authority > 12) return true;
  return false;
}

extern "C" int yrwi_query_batch(yrwi_ctx* ctx, const yrwi_query_desc* q, int32_t nq, int32_t kmax, yrwi_hit* out,
                                int32_t* nout, yrwi_stats* st) {
  if (int rc = check_batch_args(ctx, q, nq, kmax, out, nout)) return rc;
  if (nq == 0) {
    if (st) std::memset(st, 0, sizeof(*st));
    return 0;
  }
  hipSetDevice(ctx->device);
  drain(ctx);
  if (int rc = ensure_url_ids(ctx)) return rc;
  if (wants_authority(q, nq))
    if (int rc = ensure_host_ids(ctx)) return rc;
  const int64_t t0 = now_ns();
  // contiguous parts of equal query count, one per lane, each planned and run
  // by its lane's thread (every rank splits a sharded batch identically)
  const int nl = (int)std::min<int64_t>((int64_t)ctx->lanes.size(), nq);
  std::vector<yrwi_stats> pst((size_t)nl);
  for (auto& p : pst) std::memset(&p, 0, sizeof(p));
  auto cut = [&](int l) { return (int32_t)((int64_t)nq * l / nl); };
  const int64_t seq0 = ctx->coll_seq;  // collective order of the parts (CollTurn)
  ctx->coll_seq += nl;
  for (int l = 0; l < nl; l++) {
    ctx->lanes[(size_t)l]->seq = seq0 + l;
    ctx->lanes[(size_t)l]->xcall = 0;
    ctx->lanes[(size_t)l]->dcall = 0;
  }
  auto part = [=, &pst](int l) {
    Lane* L = ctx->lanes[(size_t)l];
    L->rc = run_batch_part(ctx, L, q + cut(l), cut(l + 1) - cut(l), kmax, out + (size_t)cut(l) * kmax, nout + cut(l),
                           st ? &pst[(size_t)l] : nullptr);
  };
  for (int l = 1; l < nl; l++) ctx->lanes[(size_t)l]->submit([=] { part(l); });
  part(0);  // lane 0 on the calling thread (its worker is idle after drain)
  int rc = 0;
  for (int l = 0; l < nl; l++) {
    Lane* L = ctx->lanes[(size_t)l];
    if (l > 0) L->wait();
    if (L->rc && !rc) rc = ctx->take(L, L->rc);
  }
  if (rc) return rc;
  if (st) {
    std::memset(st, 0, sizeof(*st));
    for (const yrwi_stats& p : pst) {
      st->postings_in += p.postings_in;
      st->joined += p.joined;
      st->bytes_alg += p.bytes_alg;
      st->bytes_join += p.bytes_join;
      st->bytes_probe += p.bytes_probe;
      st->bytes_probe_loaded += p.bytes_probe_loaded;
      st->bytes_probe_capped += p.bytes_probe_capped;
      st->bytes_features += p.bytes_features;
      st->bytes_join_capped += p.bytes_join_capped;
      st->bytes_alg_capped += p.bytes_alg_capped;
      st->t_join_ns += p.t_join_ns;
      st->t_probe_ns += p.t_probe_ns;
      st->bytes_compact += p.bytes_compact;
      st->t_compact_ns += p.t_compact_ns;
      st->t_kernels_ns += p.t_kernels_ns;
      st->t_norm_ns += p.t_norm_ns;
      st->t_score_ns += p.t_score_ns;
      st->n_join_launches += p.n_join_launches;
      st->n_enum_steps += p.n_enum_steps;
      st->n_test_steps += p.n_test_steps;
      st->n_realloc += p.n_realloc;
      st->n_probe_dispatches += p.n_probe_dispatches;
      st->t_probe_all_ns += p.t_probe_all_ns;
      st->n_rank_passes += p.n_rank_passes;
      st->t_reduce_ns += p.t_reduce_ns;
      st->t_scorek_ns += p.t_scorek_ns;
      st->bytes_reduce += p.bytes_reduce;
      st->bytes_score += p.bytes_score;
      st->n_chain_launches += p.n_chain_launches;
      st->t_chain_ns += p.t_chain_ns;
      st->bytes_chain += p.bytes_chain;
    }
    st->t_total_ns = now_ns() - t0;
  }
  return 0;
}

extern "C" int yrwi_query_batch_submit(yrwi_ctx* ctx, const yrwi_query_desc* q, int32_t nq, int32_t kmax,
                                       yrwi_hit* out, int32_t* nout, yrwi_stats* st, int64_t* ticket) {
  if (int rc = check_batch_args(ctx, q, nq, kmax, out, nout)) return rc;
  if (!ticket) return YRWI_E_ARG;
  hipSetDevice(ctx->device);
  if (ctx->uid_dirty) {  // the index changed: nothing can be in flight (put_list drained)
    drain(ctx);
    if (int rc = ensure_url_ids(ctx)) return rc;
  }
  if (!ctx->host_ids && wants_authority(q, nq)) {  // the first authority batch since the index changed
    drain(ctx);
    if (int rc = ensure_host_ids(ctx)) return rc;
  }
  const int64_t t = ctx->next_ticket;
  Lane* L = ctx->lanes[(size_t)(t % (int64_t)ctx->lanes.size())];
  L->wait();  // the lane's previous batch (its status is already recorded)
  ctx->next_ticket++;
  L->seq = ctx->coll_seq++;  // collective order (CollTurn): submission order, the same on every rank
  L->xcall = 0;
  L->dcall = 0;
  L->submit([=] {
    if (st) std::memset(st, 0, sizeof(*st));
    const int rc = nq == 0 ? 0 : run_batch_part(ctx, L, q, nq, kmax, out, nout, st);
    turn_release(L);  // nq == 0: nothing ran, the turn passes all the same
    {
      std::lock_guard<std::mutex> lk(ctx->st_mu);
      ctx->status[t] = {rc, rc ? L->err : std::string()};
    }
    L->done = t;
  });
  *ticket = t;
  return 0;
}

extern "C" int yrwi_query_batch_wait(yrwi_ctx* ctx, int64_t ticket) {
  if (!ctx || ticket < 0 || ticket >= ctx->next_ticket) return YRWI_E_ARG;
  Lane* L = ctx->lanes[(size_t)(ticket % (int64_t)ctx->lanes.size())];
  L->wait();  // a lane runs its tickets in order; the next one is not submitted before this returns
  std::lock_guard<std::mutex> lk(ctx->st_mu);
  auto it = ctx->status.find(ticket);
  if (it == ctx->status.end()) return ctx->fail(YRWI_E_ARG, "unknown or already collected ticket");
  const int rc = it->second.first;
  if (rc) ctx->err = it->second.second;
  ctx->status.erase(it);
  return rc;
}

extern "C" int yrwi_host_alloc(yrwi_ctx* ctx, size_t bytes, void** p) {
  if (!ctx || !p || bytes == 0) return YRWI_E_ARG;
  hipSetDevice(ctx->device);
  void* h = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess) return ctx->fail(YRWI_E_NOMEM, "hipHostMalloc");
  std::lock_guard<std::mutex> lk(ctx->hostreg.mu);
  ctx->hostreg.bufs.push_back({static_cast<uint8_t*>(h), bytes});
  *p = h;
  return 0;
}

extern "C" int yrwi_host_free(yrwi_ctx* ctx, void* p) {
  if (!ctx || !p) return YRWI_E_ARG;
  drain(ctx);
  std::lock_guard<std::mutex> lk(ctx->hostreg.mu);
  auto& v = ctx->hostreg.bufs;
  for (size_t i = 0; i < v.size(); i++)
    if (v[i].first == p) {
      hipHostFree(p);
      v.erase(v.begin() + (long)i);
      return 0;
    }
  return ctx->fail(YRWI_E_ARG, "not a yrwi_host_alloc buffer");
}

extern "C" int yrwi_query(yrwi_ctx* ctx, const yrwi_query_desc* q, yrwi_hit* out, int32_t* nout, yrwi_stats* st) {
  if (!q) return YRWI_E_ARG;
  int32_t kmax = std::max<int32_t>(1, std::min<int32_t>(q->k, YRWI_MAX_K));
  return yrwi_query_batch(ctx, q, 1, kmax, out, nout, st);
}

extern "C" int yrwi_score_nodes(yrwi_ctx* ctx, const yrwi_node* nodes, int64_t n, const yrwi_profile* prof,
                                const char* language, int32_t maxdomcount, int64_t* scores) {
  if (!ctx || n < 0 || (n > 0 && (!nodes || !scores))) return YRWI_E_ARG;
  if (n == 0) return 0;
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  yrwi_profile p;
  if (prof) p = *prof; else yrwi_profile_default(&p);
  char lang[8] = {0};
  if (language) std::strncpy(lang, language, 7);  // ReferenceOrder.language (a String; longer never equals)
  if (language && std::strlen(language) > 7) std::memset(lang, 0xFF, 7);
  yrwi_node* d_nodes = arena_alloc<yrwi_node>(L, n);
  yrwi_profile* d_prof = arena_alloc<yrwi_profile>(L, 1);
  int64_t* d_sc = arena_alloc<int64_t>(L, n);
  if (!d_nodes || !d_prof || !d_sc) return ctx->fail(YRWI_E_NOMEM, "arena");
  HIPCHK(ctx, hipMemcpyAsync(d_nodes, nodes, sizeof(yrwi_node) * (size_t)n, hipMemcpyHostToDevice, L->stream));
  HIPCHK(ctx, hipMemcpyAsync(d_prof, &p, sizeof(p), hipMemcpyHostToDevice, L->stream));
  if (launch_score_nodes(d_nodes, n, d_prof, lang, maxdomcount, d_sc, L->stream))
    return ctx->fail(YRWI_E_HIP, "score_nodes launch");
  HIPCHK(ctx, hipMemcpyAsync(scores, d_sc, sizeof(int64_t) * (size_t)n, hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, lane_sync(L));
  return 0;
}

extern "C" int yrwi_join_exclude(yrwi_ctx* ctx, const uint8_t* incl, int32_t nincl, const uint8_t* excl,
                                 int32_t nexcl, int32_t max_distance, int64_t now_ms, uint8_t* rows_out,
                                 int64_t cap_rows, int64_t* m) {
  yrwi_query_desc d{};
  d.incl = incl;
  d.nincl = nincl;
  d.excl = excl;
  d.nexcl = nexcl;
  d.max_distance = max_distance;
  d.k = 1;
  d.now_ms = now_ms;
  return yrwi_term_search(ctx, &d, rows_out, cap_rows, m);
}

extern "C" int yrwi_term_search(yrwi_ctx* ctx, const yrwi_query_desc* q, uint8_t* rows_out, int64_t cap_rows,
                                int64_t* m) {
  if (!ctx || !m || !q) return YRWI_E_ARG;
  *m = 0;
  hipSetDevice(ctx->device);
  yrwi_query_desc d = *q;
  d.k = 1;
  d.filter = nullptr;
  drain(ctx);
  if (int rc0 = ensure_url_ids(ctx)) return rc0;
  Lane* L = ctx->lanes[0];
  std::vector<Plan> plans(1);
  int rc = ctx->take(L, plan_query(ctx, L, d, &plans[0]));
  if (rc) return rc;
  if ((rc = ctx->take(L, resolve_selections(L, plans)))) return rc;
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  if ((rc = ctx->take(L, plan_batch(L, plans)))) return rc;
  rc = ctx->take(L, run_join_phase(L, plans, nullptr, nullptr));
  if (rc) return rc;
  const Plan& P = plans[0];
  if (P.empty || P.cont.n == 0) {
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
  }
  std::vector<uint8_t> rows((size_t)P.cont.n * 40), rem;
  const uint8_t* src = P.cont.rows;  // a single include list is returned as it is stored (:355-370)
  if (!src) {  // a joined container: its rows as toRowEntry re-encodes them (J6)
    uint8_t* d_rows = arena_alloc<uint8_t>(L, P.cont.n * 40);
    if (!d_rows) return ctx->fail(YRWI_E_NOMEM, "arena");
    if (launch_feat_rows(P.cont.feat, P.cont.uid, ctx->dkhi, ctx->dklo, P.cont.n, plans[0].now_ms, d_rows, L->stream))
      return ctx->fail(YRWI_E_HIP, "row launch");
    src = d_rows;
  }
  HIPCHK(ctx, hipMemcpyAsync(rows.data(), src, rows.size(), hipMemcpyDeviceToHost, ctx->stream));
  if (P.removed) {
    rem.resize((size_t)P.cont.n);
    HIPCHK(ctx, hipMemcpyAsync(rem.data(), P.removed, rem.size(), hipMemcpyDeviceToHost, ctx->stream));
  }
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  int64_t k = 0;
  for (int64_t i = 0; i < P.cont.n; i++) {
    if (!rem.empty() && rem[(size_t)i]) continue;
    if (k >= cap_rows) return ctx->fail(YRWI_E_ARG, "rows_out capacity too small");
    std::memcpy(rows_out + k * 40, rows.data() + i * 40, 40);
    k++;
  }
  *m = k;
  return 0;
}

extern "C" int yrwi_normalize_score(yrwi_ctx* ctx, const uint8_t* rows40, int64_t m, const yrwi_profile* prof,
                                    const char* language, int64_t now_ms, int64_t* score_out) {
  if (!ctx || (m > 0 && (!rows40 || !score_out))) return YRWI_E_ARG;
  if (m <= 0) return 0;
  if (m > MAX_LIST) return ctx->fail(YRWI_E_LIMIT, "container longer than 53,687,091 rows");
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  uint8_t* rows = arena_alloc<uint8_t>(L, m * 40);
  uint64_t* khi = arena_alloc<uint64_t>(L, m);
  uint8_t* klo = arena_alloc<uint8_t>(L, m);
  int32_t* derr = arena_alloc<int32_t>(L, 1);
  if (!rows || !khi || !klo || !derr) return ctx->fail(YRWI_E_NOMEM, "arena");
  HIPCHK(ctx, hipMemcpyAsync(rows, rows40, (size_t)m * 40, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync(derr, 0, 4, ctx->stream));
  if (launch_validate_rows(rows, m, khi, klo, derr, ctx->stream)) return ctx->fail(YRWI_E_HIP, "validate launch");
  int32_t herr = 0;
  HIPCHK(ctx, hipMemcpyAsync(&herr, derr, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  if (herr & 1) return ctx->fail(YRWI_E_HASH, "url hash is not well-formed Base64");
  if (herr & 2) return ctx->fail(YRWI_E_NULL_LANGUAGE, "row with empty language cell (reference NPE)");
  if (herr & 4) return ctx->fail(YRWI_E_UNSORTED, "container rows are not strictly ascending by url hash");
  std::vector<Plan> plans(1);
  Plan& P = plans[0];
  P.empty = false;
  uint64_t* feat = arena_alloc<uint64_t>(L, m * FEAT_WORDS);
  if (!feat) return ctx->fail(YRWI_E_NOMEM, "arena");
  if (launch_features(rows, m, feat, ctx->stream)) return ctx->fail(YRWI_E_HIP, "features launch");
  P.cont = DList{khi, klo, rows, m, nullptr, feat};
  P.removed = nullptr;
  if (prof) P.prof = *prof; else yrwi_profile_default(&P.prof);
  size_t ll = language ? strnlen(language, 8) : 0;
  P.lang_ok = ll == 2;
  P.lang[0] = ll > 0 ? (uint8_t)language[0] : 0;
  P.lang[1] = ll > 1 ? (uint8_t)language[1] : 0;
  P.now_ms = now_ms != 0 ? now_ms
                         : (int64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
                               std::chrono::system_clock::now().time_since_epoch()).count();
  P.k = 1;
  return ctx->take(L, run_rank_phase(L, plans, 1, nullptr, nullptr, score_out, nullptr, nullptr, false));
}
