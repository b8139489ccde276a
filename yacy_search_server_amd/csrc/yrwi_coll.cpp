// yrwi_coll.cpp -- collectives between the url-hash shards of one query batch.
//
// Production transport: RCCL over xGMI (one communicator per lane; the payloads
// are normalisation summaries, host counts and top-k lists, all latency-bound).
// Test transport: an in-process "loopback" group -- several shard contexts of
// one process on ONE GPU (RCCL refuses two ranks on one device), exchanging
// through device-to-device copies ordered by events across the ranks' streams.
// It exists so the sharded path (summary exchange, host-count owner exchange,
// shard merge) runs bit-exact tests on a one-GPU box; it is selected only by a
// group id carrying LOOP_TAG.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "yrwi_host.h"

namespace yrwi {

struct LoopGroup {
  int world = 0, members = 0;
  std::string key;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  int64_t gen = 0;
  struct Post {
    const void* send = nullptr;
    size_t bytes = 0;
    std::vector<Xfer> sends;
    hipEvent_t ready = nullptr, done = nullptr;
  };
  std::vector<Post> posts;

  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const int64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

static std::mutex g_loop_mu;
static std::map<std::string, LoopGroup*> g_loops;

LoopGroup* loop_join(const uint8_t id[128], int world, int rank) {
  std::lock_guard<std::mutex> lk(g_loop_mu);
  std::string key(reinterpret_cast<const char*>(id), 128);
  LoopGroup*& g = g_loops[key];
  if (!g) {
    g = new LoopGroup();
    g->world = world;
    g->key = key;
    g->posts.resize((size_t)world);
  }
  if (g->world != world || rank < 0 || rank >= world) return nullptr;
  g->members++;
  return g;
}

void loop_leave(LoopGroup* g) {
  std::lock_guard<std::mutex> lk(g_loop_mu);
  if (--g->members == 0) {
    g_loops.erase(g->key);
    delete g;
  }
}

static int ensure_events(Lane* L) {
  for (auto& e : L->coll_ev)
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return L->fail(YRWI_E_HIP, "event");
  return 0;
}

// Loopback round: post (ready event), barrier, run `copy` after every peer's
// ready event, post done, barrier, wait for every peer's done event (so nobody
// rewrites a buffer another rank still reads), barrier (posts reusable).
template <class F>
static int loop_round(Lane* L, const void* send, size_t bytes, const std::vector<Xfer>* sends, F copy) {
  LoopGroup* g = L->loop;
  if (ensure_events(L)) return YRWI_E_HIP;
  LoopGroup::Post& me = g->posts[(size_t)L->rank];
  me.send = send;
  me.bytes = bytes;
  if (sends) me.sends = *sends; else me.sends.clear();
  if (hipEventRecord(L->coll_ev[0], L->stream) != hipSuccess) return L->fail(YRWI_E_HIP, "event record");
  me.ready = L->coll_ev[0];
  g->barrier();
  for (auto& p : g->posts)
    if (hipStreamWaitEvent(L->stream, p.ready, 0) != hipSuccess) return L->fail(YRWI_E_HIP, "stream wait");
  int rc = copy(g);
  if (hipEventRecord(L->coll_ev[1], L->stream) != hipSuccess) return L->fail(YRWI_E_HIP, "event record");
  me.done = L->coll_ev[1];
  g->barrier();
  for (auto& p : g->posts)
    if (hipStreamWaitEvent(L->stream, p.done, 0) != hipSuccess) return L->fail(YRWI_E_HIP, "stream wait");
  g->barrier();
  return rc;
}

void turn_acquire(Lane* L) {
  if (!L->turn || L->seq < 0 || L->turn_held) return;
  std::unique_lock<std::mutex> lk(L->turn->mu);
  L->turn->cv.wait(lk, [L] { return L->turn->next == L->seq; });
  L->turn_held = true;
}

void turn_release(Lane* L) {
  if (!L->turn || L->seq < 0 || !L->sharded) {  // one context: no collectives to order
    L->seq = -1;
    return;
  }
  {
    std::unique_lock<std::mutex> lk(L->turn->mu);
    // a part that never held the turn still passes it, in order
    L->turn->cv.wait(lk, [L] { return L->turn->next == L->seq; });
    L->turn->next = L->seq + 1;
  }
  L->turn->cv.notify_all();
  L->seq = -1;
  L->turn_held = false;
}

// ---------------------------------------------------------------- host exchange
// The batch's global list sizes (J1/J2/J3 planning) are host data: the ranks of
// one node sum them through a shared-memory mailbox instead of a device
// collective.  A mailbox exchange waits only for the same batch part on the
// other ranks, never for a device queue, so it needs no collective turn: the
// parts' planning and joins overlap freely and the turn (CollTurn) is held only
// around the rank phase's device collectives.  One exchange = one key (part
// sequence number * HX_CALLS + call index, identical on every rank); a slot is
// claimed by the first rank to reach its key, written by every rank, read by
// every rank and freed by the last reader.  Longer vectors, unordered callers
// and a missing mailbox fall back to the device all-gather.
namespace {
constexpr int HX_SLOTS = 64, HX_MAXN = 4096, HX_CALLS = 8, HX_MAXW = 16, HX_ABORTS = 64;
struct HxEntry {
  int64_t n;
  int64_t v[HX_MAXN];
};
// One slot's whole state in one word, every transition a compare-and-swap:
// (key + 1) << 16 | writers << 8 | leavers (0: free).  A rank joins the slot of
// its key, writes its entry, counts itself among the writers, waits for all
// `world` writers, reads, and leaves; the last to leave frees the slot.  A rank
// that gives up (its part's sequence was aborted) leaves as well, so the slot of
// an aborted exchange is freed once every rank that wrote to it has left.
struct HxSlot {
  std::atomic<uint64_t> state;
  char pad[56];
};
}  // namespace

// segment header: ranks that mapped it (the last of `world` unlinks the name);
// aborted[seq % HX_ABORTS] = seq + 1: that batch part failed on some rank, and
// every rank's waits on that part's exchanges give up at once (its peers would
// otherwise each hold a core for the whole timeout per exchange).  Only that
// part: the exchanges of every later part run as usual.
struct HxHead {
  std::atomic<int32_t> attached;
  int32_t pad0;
  std::atomic<int64_t> aborted[HX_ABORTS];
  // device identity of every rank (hostx_device_peers): PCI domain / bus / device + 1, 0 = not yet posted
  std::atomic<int64_t> devid[HX_MAXW];
  char pad[56];
};

struct HostX {
  void* base = nullptr;
  size_t bytes = 0;
  int world = 0, rank = 0;
  std::string name;
  HxHead* head() const { return static_cast<HxHead*>(base); }
  HxSlot* slot(int i) const {
    return reinterpret_cast<HxSlot*>(static_cast<char*>(base) + sizeof(HxHead) + (size_t)i * sizeof(HxSlot));
  }
  HxEntry* entry(int i, int r) const {
    char* e0 = static_cast<char*>(base) + sizeof(HxHead) + (size_t)HX_SLOTS * sizeof(HxSlot);
    return reinterpret_cast<HxEntry*>(e0 + ((size_t)i * world + r) * sizeof(HxEntry));
  }
  bool aborted(int64_t seq) const {
    return seq >= 0 && head()->aborted[seq % HX_ABORTS].load(std::memory_order_acquire) == seq + 1;
  }
};

HostX* hostx_open(const uint8_t id[128], int world, int rank) {
  if (world < 2 || world > HX_MAXW || getenv("YRWI_NO_HOSTX")) return nullptr;
  uint64_t h = 1469598103934665603ull;  // FNV-1a of the group id: the segment's name
  for (int i = 0; i < 128; i++) h = (h ^ id[i]) * 1099511628211ull;
  char nm[64];
  snprintf(nm, sizeof(nm), "/yrwi-hx-%016llx-%d", (unsigned long long)h, world);
  const size_t bytes =
      sizeof(HxHead) + (size_t)HX_SLOTS * sizeof(HxSlot) + (size_t)HX_SLOTS * world * sizeof(HxEntry);
  const int fd = shm_open(nm, O_CREAT | O_RDWR, 0600);  // zero-filled when new: every slot free
  if (fd < 0) return nullptr;
  if (ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  HostX* x = new HostX();
  x->base = p;
  x->bytes = bytes;
  x->world = world;
  x->rank = rank;
  x->name = nm;
  // every rank of the group maps the segment before its first exchange (at
  // open); the last one to do so removes the name, so nothing is left in
  // /dev/shm whatever way the processes end
  if (x->head()->attached.fetch_add(1, std::memory_order_acq_rel) + 1 == world) shm_unlink(nm);
  return x;
}

int hostx_attached(const HostX* x) { return x ? x->head()->attached.load(std::memory_order_acquire) : 0; }

// wait (up to limit_s) until every rank of the group mapped the mailbox; false on timeout
bool hostx_wait_attached(const HostX* x, double limit_s) {
  if (!x) return false;
  const auto t0 = std::chrono::steady_clock::now();
  while (hostx_attached(x) < x->world) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  return true;
}

// Posts this rank's device identity and waits (up to limit_s) for every rank's.
// Returns how many other ranks of the group run on the same device (PCI domain,
// bus and device equal), or -1 when some rank never posted.  Every rank reads the
// same table, so all of them reach the same answer.
int hostx_device_peers(const HostX* x, int64_t my_devid, double limit_s) {
  if (!x) return -1;
  HxHead* h = x->head();
  h->devid[x->rank].store(my_devid, std::memory_order_release);
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    int posted = 0, same = 0;
    for (int r = 0; r < x->world; r++) {
      const int64_t d = h->devid[r].load(std::memory_order_acquire);
      posted += d != 0;
      same += r != x->rank && d == my_devid;
    }
    if (posted == x->world) return same;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) return -1;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

void hostx_abort(HostX* x, int64_t seq) {
  if (x && seq >= 0) x->head()->aborted[seq % HX_ABORTS].store(seq + 1, std::memory_order_release);
}

void hostx_close(HostX* x, bool unlink_name) {
  if (!x) return;
  munmap(x->base, x->bytes);
  if (unlink_name) shm_unlink(x->name.c_str());
  delete x;
}

// spin, then yield; false once batch part `seq` is aborted, or after
// YRWI_HOSTX_TIMEOUT_S (default 300 s: a peer that never arrives fails the batch
// instead of hanging it; a peer busy rebuilding its url dictionary arrives late)
template <class F>
static bool hx_wait(const HostX* x, int64_t seq, F ready) {  // (x may be null: no abort table)
  static const double limit_s = getenv("YRWI_HOSTX_TIMEOUT_S") ? atof(getenv("YRWI_HOSTX_TIMEOUT_S")) : 300.0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int64_t i = 0;; i++) {
    if (ready()) return true;
    if (x && x->aborted(seq)) return false;
    if (i < 2000) {
      __builtin_ia32_pause();
      continue;
    }
    sched_yield();
    if ((i & 1023) == 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s)
      return false;
  }
}

// leave the slot of `key` (read it, or gave up after writing to it); the last
// leaver frees it: all `world` ranks read it, or its part was aborted and every
// rank that wrote to it has left
static void hx_leave(const HostX* x, HxSlot* S, int64_t key, int64_t seq) {
  uint64_t cur = S->state.load(std::memory_order_acquire);
  while ((int64_t)(cur >> 16) == key + 1) {
    const uint64_t nw = (cur >> 8) & 0xFF, nr = (cur & 0xFF) + 1;
    const bool free_it = nr == (uint64_t)x->world || (nr >= nw && x->aborted(seq));
    if (S->state.compare_exchange_weak(cur, free_it ? 0 : cur + 1, std::memory_order_acq_rel)) return;
  }
}

// 1: not handled here (caller falls back to the device all-gather); <0: error
int hostx_allsum(Lane* L, std::vector<int64_t>& v) {
  HostX* x = L->hostx;
  if (!x || L->seq < 0 || L->xcall >= HX_CALLS || v.size() > (size_t)HX_MAXN) return 1;
  const int64_t seq = L->seq, key = seq * HX_CALLS + L->xcall++;
  const uint64_t tag = (uint64_t)(key + 1) << 16;
  const int si = (int)(key % HX_SLOTS);
  HxSlot* S = x->slot(si);
  auto gave_up = [&](const char* why) {
    return L->fail(YRWI_E_RCCL, x->aborted(seq) ? "host exchange: a peer's batch part failed" : why);
  };
  // claim (or join) the slot for this key
  if (!hx_wait(x, seq, [&] {
        uint64_t cur = S->state.load(std::memory_order_acquire);
        if ((cur >> 16) == tag >> 16) return true;
        if (cur != 0) return false;
        return S->state.compare_exchange_strong(cur, tag, std::memory_order_acq_rel) || (cur >> 16) == tag >> 16;
      }))
    return gave_up("host exchange: slot never freed");
  HxEntry* me = x->entry(si, x->rank);
  me->n = (int64_t)v.size();
  std::memcpy(me->v, v.data(), v.size() * sizeof(int64_t));
  // count this write, unless the slot was freed meanwhile (the part was aborted)
  uint64_t cur = S->state.load(std::memory_order_acquire);
  do {
    if ((cur >> 16) != tag >> 16) return gave_up("host exchange: slot lost");
  } while (!S->state.compare_exchange_weak(cur, cur + (1u << 8), std::memory_order_acq_rel));
  if (!hx_wait(x, seq, [&] {
        const uint64_t s = S->state.load(std::memory_order_acquire);
        return (s >> 16) == tag >> 16 && ((s >> 8) & 0xFF) == (uint64_t)x->world;
      })) {
    hx_leave(x, S, key, seq);
    return gave_up("host exchange: a rank never arrived");
  }
  std::vector<int64_t> sum(v.size(), 0);
  int rc = 0;
  for (int r = 0; r < x->world && !rc; r++) {
    const HxEntry* e = x->entry(si, r);
    if (e->n != (int64_t)v.size()) rc = L->fail(YRWI_E_RCCL, "host exchange: size mismatch");
    for (size_t i = 0; i < v.size() && !rc; i++) sum[i] += e->v[i];
  }
  hx_leave(x, S, key, seq);
  if (rc) return rc;
  v.swap(sum);
  return 0;
}

}  // namespace yrwi

extern "C" int yrwi_hostx_selftest(const uint8_t id[128], int world, int rank, int64_t nparts, int32_t ncalls,
                                   int64_t n) {
  using namespace yrwi;
  HostX* x = hostx_open(id, world, rank);
  if (!x) return 1;
  // n < 0: the last rank's first batch part fails before its exchanges (it aborts
  // that part, as run_batch_part does): every other rank's part 0 must fail fast,
  // and every later part must then run normally on every rank.  Returns part 0's
  // status when the later parts all succeed, 1000 + the failing part otherwise.
  const bool fail_last = n < 0;
  if (fail_last) n = -n;
  Lane L;  // host-side state only: no stream, no worker thread
  L.world = world;
  L.rank = rank;
  L.hostx = x;
  int rc = 0, rc0 = 0;
  for (int64_t p = 0; p < nparts; p++) {
    L.seq = p;
    L.xcall = 0;
    int prc = 0;
    if (fail_last && p == 0 && rank == world - 1) {
      hostx_abort(x, p);
      prc = YRWI_E_RCCL;
    }
    for (int32_t c = 0; c < ncalls && prc == 0; c++) {
      std::vector<int64_t> v((size_t)n);
      for (int64_t i = 0; i < n; i++) v[(size_t)i] = rank + p + c + i;
      const int r = hostx_allsum(&L, v);
      if (r != 0) { prc = r < 0 ? r : YRWI_E_RCCL; break; }
      for (int64_t i = 0; i < n; i++)
        if (v[(size_t)i] != (int64_t)world * (p + c + i) + (int64_t)world * (world - 1) / 2) { prc = YRWI_E_RCCL; break; }
    }
    if (prc && fail_last && p == 0) {
      hostx_abort(x, p);
      rc0 = prc;
      continue;
    }
    if (prc) {
      rc = fail_last ? 1000 + (int)p : prc;
      break;
    }
  }
  if (!rc && fail_last) rc = rc0;
  hostx_close(x, rank == 0);
  return rc;
}

namespace yrwi {

// ------------------------------------------------- host-staged device collectives
// When RCCL cannot form the group -- several ranks on ONE device (RCCL refuses a
// duplicate GPU), as on a one-GPU test box -- the shards of one node exchange the
// rank phase's device buffers (ShardSum all-gather, host-count exchange, flag
// counts, top-k all-gather) through a shared-memory segment instead: each rank
// copies its payload into its region, and reads its peers' regions once all have
// posted the round.  The collective turn (CollTurn) already orders every device
// collective of a rank in one total order, the same on every rank, so one round
// is in progress at a time; a round is keyed by (batch part, call), and peers'
// `posted` / `done` words are compared for equality with that key (a peer can be
// at most one round behind).  Synchronous with the lane's stream; latency, not
// bandwidth, is what it costs -- it is the transport of the multi-process tests
// on one GPU, not of the 8-GPU node (RCCL over xGMI).
namespace {
constexpr int DX_MAXW = 16, DX_MAXE = 64;
struct DxEnt {
  int32_t peer;  // destination rank, -1: every rank (all-gather)
  int32_t pad;
  uint64_t off, bytes;
};
struct DxRank {
  std::atomic<int64_t> posted;  // key of the round whose payload is in place
  std::atomic<int64_t> done;    // key of the round this rank has finished reading
  int32_t nent, pad;
  DxEnt ent[DX_MAXE];
  char pad2[48];
};
struct DxHead {
  std::atomic<int32_t> attached;
  int32_t pad;
  std::atomic<uint64_t> cap;  // payload bytes per rank, set by the first rank to attach
  char pad2[48];
  DxRank r[DX_MAXW];
};
}  // namespace

struct DevX {
  void* base = nullptr;
  size_t bytes = 0, cap = 0;  // segment size; payload bytes per rank
  int world = 0, rank = 0;
  std::string name;
  HostX* hx = nullptr;  // abort table of the batch parts (hostx_abort)
  int64_t unordered = 0;
  DxHead* head() const { return static_cast<DxHead*>(base); }
  uint8_t* region(int r) const {
    return static_cast<uint8_t*>(base) + ((sizeof(DxHead) + 4095) & ~(size_t)4095) + (size_t)r * cap;
  }
};

DevX* devx_open(const uint8_t id[128], int world, int rank, HostX* hx) {
  if (world < 2 || world > DX_MAXW || !hx) return nullptr;
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < 128; i++) h = (h ^ id[i]) * 1099511628211ull;
  char nm[64];
  snprintf(nm, sizeof(nm), "/yrwi-dx-%016llx-%d", (unsigned long long)h, world);
  // payload bytes per rank (YRWI_DEVX_MB, default 256): the largest round is the
  // host-count exchange (12 B per distinct (query, host) of the part); untouched
  // pages of the segment cost nothing
  const char* e = getenv("YRWI_DEVX_MB");
  const size_t cap = (size_t)((e ? atof(e) : 256.0) * (double)(1 << 20) + 4095) & ~(size_t)4095;
  const size_t bytes = ((sizeof(DxHead) + 4095) & ~(size_t)4095) + (size_t)world * cap;
  const int fd = shm_open(nm, O_CREAT | O_RDWR, 0600);
  if (fd < 0) return nullptr;
  // the segment is sparse: a tmpfs smaller than it would raise SIGBUS on a later
  // write instead of an error here, so its free space must cover every region
  struct statvfs fs;
  if (fstatvfs(fd, &fs) != 0 || (uint64_t)fs.f_bavail * fs.f_frsize < (uint64_t)bytes) {
    fprintf(stderr, "yrwi: host-staged collectives need %zu MB of /dev/shm (YRWI_DEVX_MB x ranks)\n",
            bytes >> 20);
    close(fd);
    return nullptr;
  }
  if (ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  // every rank must place the regions alike: the first to attach records its
  // payload size, the others must have the same (YRWI_DEVX_MB differs otherwise)
  uint64_t want = 0;
  DxHead* hd = static_cast<DxHead*>(p);
  if (!hd->cap.compare_exchange_strong(want, (uint64_t)cap, std::memory_order_acq_rel) && want != (uint64_t)cap) {
    fprintf(stderr, "yrwi: host-staged collectives: YRWI_DEVX_MB differs between ranks (%llu vs %zu bytes)\n",
            (unsigned long long)want, cap);
    hd->attached.fetch_add(1, std::memory_order_acq_rel);
    munmap(p, bytes);
    return nullptr;
  }
  DevX* x = new DevX();
  x->base = p;
  x->bytes = bytes;
  x->cap = cap;
  x->world = world;
  x->rank = rank;
  x->name = nm;
  x->hx = hx;
  // posted / done start at the "no round" key (a new segment is zero-filled, and
  // keys are never 0: see dx_key)
  if (x->head()->attached.fetch_add(1, std::memory_order_acq_rel) + 1 == world) shm_unlink(nm);
  return x;
}

void devx_close(DevX* x, bool unlink_name) {
  if (!x) return;
  munmap(x->base, x->bytes);
  if (unlink_name) shm_unlink(x->name.c_str());
  delete x;
}

// the round's key: (batch part, call) -- never 0, so a fresh segment's zeros
// match no round; unordered callers (no part sequence) count apart
static int64_t dx_key(Lane* L) {
  if (L->seq >= 0) return ((L->seq + 1) << 8) | (int64_t)(L->dcall++ & 0xFF);
  return -(++L->devx->unordered);
}

// One round: my payload (entries to peers) into my region, wait until every rank
// posted this key, `take` copies what is mine out of the peers' regions, then
// signal done and wait until every rank has read (my region is reused next round).
template <class F>
static int dx_round(Lane* L, const std::vector<Xfer>& sends, bool all, F take) {
  DevX* x = L->devx;
  const int64_t key = dx_key(L), seq = L->seq;
  DxRank& me = x->head()->r[x->rank];
  auto gave_up = [&](const char* why) {
    return L->fail(YRWI_E_RCCL, x->hx && x->hx->aborted(seq) ? "host-staged collective: a peer's batch part failed"
                                                              : why);
  };
  HIPCHK(L, lane_sync(L));  // the payloads are complete
  uint64_t off = 0;
  int32_t ne = 0;
  for (const Xfer& s : sends) {
    if (ne == DX_MAXE) return L->fail(YRWI_E_RCCL, "host-staged collective: too many peers");
    if (off + s.bytes > x->cap)
      return L->fail(YRWI_E_RCCL, "host-staged collective: payload above YRWI_DEVX_MB per rank");
    if (s.bytes) HIPCHK(L, hipMemcpy(x->region(x->rank) + off, s.ptr, s.bytes, hipMemcpyDeviceToHost));
    me.ent[ne++] = DxEnt{all ? -1 : s.peer, 0, off, s.bytes};
    off += (s.bytes + 255) & ~(uint64_t)255;
  }
  me.nent = ne;
  me.posted.store(key, std::memory_order_release);
  if (!hx_wait(x->hx, seq, [&] {
        for (int r = 0; r < x->world; r++)
          if (x->head()->r[r].posted.load(std::memory_order_acquire) != key) return false;
        return true;
      }))
    return gave_up("host-staged collective: a rank never arrived");
  int rc = take(x);
  if (!rc && lane_sync(L) != hipSuccess) rc = L->fail(YRWI_E_HIP, "host-staged collective: copy");
  me.done.store(key, std::memory_order_release);
  if (!hx_wait(x->hx, seq, [&] {
        for (int r = 0; r < x->world; r++)
          if (x->head()->r[r].done.load(std::memory_order_acquire) != key) return false;
        return true;
      }))
    return rc ? rc : gave_up("host-staged collective: a rank never finished reading");
  return rc;
}

static int dx_allgather(Lane* L, const void* send, void* recv, size_t bytes) {
  return dx_round(L, {Xfer{-1, const_cast<void*>(send), bytes}}, true, [&](DevX* x) {
    for (int p = 0; p < x->world; p++) {
      const DxRank& q = x->head()->r[p];
      if (q.nent != 1 || q.ent[0].bytes != bytes) return L->fail(YRWI_E_RCCL, "host-staged all-gather: size mismatch");
      if (bytes && hipMemcpyAsync(static_cast<uint8_t*>(recv) + (size_t)p * bytes, x->region(p) + q.ent[0].off, bytes,
                                  hipMemcpyHostToDevice, L->stream) != hipSuccess)
        return L->fail(YRWI_E_HIP, "host-staged all-gather: copy");
    }
    return 0;
  });
}

static int dx_exchange(Lane* L, const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs) {
  return dx_round(L, sends, false, [&](DevX* x) {
    for (const Xfer& rv : recvs) {
      if (!rv.bytes) continue;
      const DxRank& q = x->head()->r[rv.peer];
      const DxEnt* src = nullptr;
      for (int i = 0; i < q.nent; i++)
        if (q.ent[i].peer == L->rank && q.ent[i].bytes) src = &q.ent[i];
      if (!src || src->bytes != rv.bytes) return L->fail(YRWI_E_RCCL, "host-staged exchange: unmatched receive");
      if (hipMemcpyAsync(rv.ptr, x->region(rv.peer) + src->off, rv.bytes, hipMemcpyHostToDevice, L->stream) !=
          hipSuccess)
        return L->fail(YRWI_E_HIP, "host-staged exchange: copy");
    }
    return 0;
  });
}

int coll_allgather(Lane* L, const void* send, void* recv, size_t bytes) {
  if (L->sharded) turn_acquire(L);
  if (!L->sharded) {
    if (hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, L->stream) != hipSuccess)
      return L->fail(YRWI_E_HIP, "copy");
    return 0;
  }
  if (L->devx) return dx_allgather(L, send, recv, bytes);
  if (!L->loop) {
    if (ncclAllGather(send, recv, bytes, ncclChar, L->comm, L->stream) != ncclSuccess)
      return L->fail(YRWI_E_RCCL, "allgather");
    return 0;
  }
  return loop_round(L, send, bytes, nullptr, [&](LoopGroup* g) {
    for (int p = 0; p < g->world; p++) {
      const LoopGroup::Post& q = g->posts[(size_t)p];
      if (q.bytes != bytes) return L->fail(YRWI_E_RCCL, "loopback allgather: size mismatch");
      if (bytes && hipMemcpyAsync(static_cast<uint8_t*>(recv) + (size_t)p * bytes, q.send, bytes,
                                  hipMemcpyDeviceToDevice, L->stream) != hipSuccess)
        return L->fail(YRWI_E_HIP, "loopback copy");
    }
    return 0;
  });
}

int coll_allreduce_i32(Lane* L, int32_t* buf, size_t n, bool max_op) {
  if (!L->sharded || n == 0) return 0;
  turn_acquire(L);
  if (!L->loop && !L->devx) {
    if (ncclAllReduce(buf, buf, n, ncclInt32, max_op ? ncclMax : ncclSum, L->comm, L->stream) != ncclSuccess)
      return L->fail(YRWI_E_RCCL, "allreduce");
    return 0;
  }
  int32_t* all = reinterpret_cast<int32_t*>(L->arena.alloc(n * 4 * (size_t)L->world));
  if (!all) return L->fail(YRWI_E_NOMEM, "arena");
  if (int rc = coll_allgather(L, buf, all, n * 4)) return rc;
  if (launch_reduce_i32(all, L->world, (int64_t)n, buf, max_op ? 1 : 0, L->stream)) return L->fail(YRWI_E_HIP, "reduce");
  return 0;
}

int coll_exchange(Lane* L, const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs) {
  turn_acquire(L);
  if (L->devx) return dx_exchange(L, sends, recvs);
  if (!L->loop) {
    if (ncclGroupStart() != ncclSuccess) return L->fail(YRWI_E_RCCL, "group");
    for (const Xfer& x : sends)
      if (x.bytes && ncclSend(x.ptr, x.bytes, ncclChar, x.peer, L->comm, L->stream) != ncclSuccess)
        return L->fail(YRWI_E_RCCL, "send");
    for (const Xfer& x : recvs)
      if (x.bytes && ncclRecv(x.ptr, x.bytes, ncclChar, x.peer, L->comm, L->stream) != ncclSuccess)
        return L->fail(YRWI_E_RCCL, "recv");
    if (ncclGroupEnd() != ncclSuccess) return L->fail(YRWI_E_RCCL, "group end");
    return 0;
  }
  return loop_round(L, nullptr, 0, &sends, [&](LoopGroup* g) {
    for (const Xfer& x : recvs) {
      if (!x.bytes) continue;
      const Xfer* src = nullptr;
      for (const Xfer& y : g->posts[(size_t)x.peer].sends)
        if (y.peer == L->rank && y.bytes) src = &y;
      if (!src || src->bytes != x.bytes) return L->fail(YRWI_E_RCCL, "loopback exchange: unmatched receive");
      if (hipMemcpyAsync(x.ptr, src->ptr, x.bytes, hipMemcpyDeviceToDevice, L->stream) != hipSuccess)
        return L->fail(YRWI_E_HIP, "loopback copy");
    }
    return 0;
  });
}

}  // namespace yrwi
