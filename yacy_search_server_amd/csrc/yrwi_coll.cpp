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

#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
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
  if (!L->turn || L->seq < 0 || L->world <= 1) {  // one context: no collectives to order
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

int coll_allgather(Lane* L, const void* send, void* recv, size_t bytes) {
  if (L->world > 1) turn_acquire(L);
  if (L->world <= 1) {
    if (hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, L->stream) != hipSuccess)
      return L->fail(YRWI_E_HIP, "copy");
    return 0;
  }
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
  if (L->world <= 1 || n == 0) return 0;
  turn_acquire(L);
  if (!L->loop) {
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
