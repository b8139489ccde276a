// yrwi_dict.hip -- the url dictionary of a context (one GPU / one url-hash shard).
//
// Every posting's url hash is replaced, for the joins, by its url id: the rank
// of the hash among all distinct url hashes of the context's lists.  Ranks
// preserve Base64Order (the 72-bit key order), so a list sorted by url hash is
// sorted by url id and every merge / probe / exclusion decision is unchanged,
// while the join kernels stream and compare 4-byte ids instead of 9-byte keys
// (DESIGN.md §3).  The dictionary is rebuilt on the device before the first
// query after any list changed: all keys are radix-sorted (klo, then stably
// khi) with their posting positions, equal neighbours share a rank, and the
// ranks are scattered back to each list's uid slice.

#include <hipcub/hipcub.hpp>

#include "yrwi_host.h"

namespace yrwi {
namespace {

struct DictSeg {
  const uint64_t* khi;
  const uint8_t* klo;
};

__global__ void k_dict_gather(const DictSeg* __restrict__ segs, const int64_t* __restrict__ off, int nseg, int64_t n,
                              uint64_t* __restrict__ kh, uint8_t* __restrict__ kl, uint32_t* __restrict__ pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int lo = 0, hi = nseg - 1;  // last segment with off <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const int64_t j = i - off[lo];
  kh[i] = segs[lo].khi[j];
  kl[i] = segs[lo].klo[j];
  pos[i] = (uint32_t)i;
}

__global__ void k_gather_u64(const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t n,
                             uint64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

// flag[j] = 1 if sorted key j differs from key j-1 (klo looked up in posting order)
__global__ void k_dict_flags(const uint64_t* __restrict__ kh, const uint32_t* __restrict__ pos,
                             const uint8_t* __restrict__ kl, int64_t n, uint32_t* __restrict__ flag) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  flag[j] = (j == 0 || kh[j] != kh[j - 1] || kl[pos[j]] != kl[pos[j - 1]]) ? 1u : 0u;
}

__global__ void k_dict_scatter(const uint32_t* __restrict__ rank1, const uint32_t* __restrict__ pos, int64_t n,
                               uint32_t* __restrict__ uid) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) uid[pos[j]] = rank1[j] - 1u;
}

// the key of every url id: the first posting of each run of equal keys
__global__ void k_dict_keys(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ rank1,
                            const uint64_t* __restrict__ kh, const uint8_t* __restrict__ kl,
                            const uint32_t* __restrict__ pos, int64_t n, uint64_t* __restrict__ dkhi,
                            uint8_t* __restrict__ dklo) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || !flag[j]) return;
  const uint32_t u = rank1[j] - 1u;
  dkhi[u] = kh[j];
  dklo[u] = kl[pos[j]];
}

unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) hipFree(p);
  }
  template <class T>
  T* get(size_t count) {
    if (hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess) p = nullptr;
    return static_cast<T*>(p);
  }
};

}  // namespace

int ensure_url_ids(CtxBase* ctx) {
  if (!ctx->uid_dirty) return 0;
  hipStream_t st = ctx->stream;
  std::vector<ListRec*> lists;
  int64_t n = 0;
  for (auto& kv : ctx->lists) {
    lists.push_back(&kv.second);
    n += kv.second.n;
  }
  if (n > (int64_t)INT32_MAX) return ctx->fail(YRWI_E_LIMIT, "more than 2^31 postings in one context");
  if (n > 0 && (size_t)n > ctx->uid_cap) {
    if (ctx->uid_all) hipFree(ctx->uid_all);
    ctx->uid_all = nullptr;
    ctx->uid_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->uid_all), (size_t)n * 4) != hipSuccess)
      return ctx->fail(YRWI_E_NOMEM, "url id allocation");
    ctx->uid_cap = (size_t)n;
  }
  if (n == 0) {
    ctx->uid_dirty = false;
    return 0;
  }
  // ranking records of lists that have none yet (new or replaced lists)
  for (ListRec* L : lists) {
    if (L->feat || L->n == 0) continue;
    L->feat = reinterpret_cast<uint64_t*>(ctx->index_mem.alloc((size_t)L->n * FEAT_BYTES));
    if (!L->feat) return ctx->fail(YRWI_E_NOMEM, "ranking record allocation");
    if (launch_features(L->rows, L->n, L->feat, st)) return ctx->fail(YRWI_E_HIP, "features launch");
  }
  std::vector<DictSeg> segs;
  std::vector<int64_t> off;
  int64_t o = 0;
  for (ListRec* L : lists) {
    segs.push_back({L->khi, L->klo});
    off.push_back(o);
    L->uid = ctx->uid_all + o;
    o += L->n;
  }
  DevBuf bsegs, boff, bkh, bkh2, bkl, bkl2, bpos, bpos2, bflag, brank, btmp;
  DictSeg* d_segs = bsegs.get<DictSeg>(segs.size());
  int64_t* d_off = boff.get<int64_t>(off.size());
  uint64_t* kh = bkh.get<uint64_t>((size_t)n);
  uint64_t* kh2 = bkh2.get<uint64_t>((size_t)n);
  uint8_t* kl = bkl.get<uint8_t>((size_t)n);
  uint8_t* kl2 = bkl2.get<uint8_t>((size_t)n);
  uint32_t* pos = bpos.get<uint32_t>((size_t)n);
  uint32_t* pos2 = bpos2.get<uint32_t>((size_t)n);
  uint32_t* flag = bflag.get<uint32_t>((size_t)n);
  uint32_t* rank1 = brank.get<uint32_t>((size_t)n);
  if (!d_segs || !d_off || !kh || !kh2 || !kl || !kl2 || !pos || !pos2 || !flag || !rank1)
    return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
  HIPCHK(ctx, hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(DictSeg), hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(d_off, off.data(), off.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
  const int ni = (int)n;
  hipLaunchKernelGGL(k_dict_gather, dim3(nb(n)), dim3(256), 0, st, d_segs, d_off, (int)segs.size(), n, kh, kl, pos);
  size_t t1 = 0, t2 = 0, t3 = 0;
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t1, kl, kl2, pos, pos2, ni, 0, 8, st));
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t2, kh2, kh, pos2, pos, ni, 0, 64, st));
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(nullptr, t3, flag, rank1, ni, st));
  size_t tb = std::max(t1, std::max(t2, t3));
  void* tmp = btmp.get<uint8_t>(tb);
  if (!tmp) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
  // (klo) then, stably, (khi): sorted by the 72-bit key; pos = posting index
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t1, kl, kl2, pos, pos2, ni, 0, 8, st));
  hipLaunchKernelGGL(k_gather_u64, dim3(nb(n)), dim3(256), 0, st, kh, pos2, n, kh2);
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t2, kh2, kh, pos2, pos, ni, 0, 64, st));
  hipLaunchKernelGGL(k_dict_flags, dim3(nb(n)), dim3(256), 0, st, kh, pos, kl, n, flag);
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(tmp, t3, flag, rank1, ni, st));
  hipLaunchKernelGGL(k_dict_scatter, dim3(nb(n)), dim3(256), 0, st, rank1, pos, n, ctx->uid_all);
  uint32_t nurls = 0;
  HIPCHK(ctx, hipMemcpyAsync(&nurls, rank1 + (n - 1), 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  if ((size_t)nurls > ctx->dict_cap) {
    if (ctx->dkhi) hipFree(ctx->dkhi);
    if (ctx->dklo) hipFree(ctx->dklo);
    ctx->dkhi = nullptr;
    ctx->dklo = nullptr;
    ctx->dict_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->dkhi), (size_t)nurls * 8) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&ctx->dklo), (size_t)nurls) != hipSuccess)
      return ctx->fail(YRWI_E_NOMEM, "url dictionary allocation");
    ctx->dict_cap = nurls;
  }
  ctx->nurls = nurls;
  for (Lane* L : ctx->lanes) {  // no batch is in flight while the dictionary is rebuilt
    L->dkhi = ctx->dkhi;
    L->dklo = ctx->dklo;
  }
  hipLaunchKernelGGL(k_dict_keys, dim3(nb(n)), dim3(256), 0, st, flag, rank1, kh, kl, pos, n, ctx->dkhi, ctx->dklo);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipStreamSynchronize(st));  // scratch is freed on return
  ctx->uid_dirty = false;
  return 0;
}

}  // namespace yrwi
