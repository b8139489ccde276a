// yrwi_dict.hip -- the url dictionary of a context (one GPU / one url-hash shard).
//
// Every posting's url hash is replaced, for the joins, by its url id: the rank
// of the hash among all distinct url hashes of the context's lists.  Ranks
// preserve Base64Order (the 72-bit key order), so a list sorted by url hash is
// sorted by url id and every merge / probe / exclusion decision is unchanged,
// while the join kernels stream and compare 4-byte ids instead of 9-byte keys
// (DESIGN.md §3).  Built in full the first time (and when much of the index
// changed): all keys are radix-sorted (klo, then stably khi) with their posting
// positions, equal neighbours share a rank, and the ranks are scattered back to
// each list's uid slice.  After that, the lists added or replaced since the last
// query are merged in incrementally (IndexCell.add keeps adding postings,
// IndexCell.java:289): only their keys are sorted; keys new to the dictionary get
// their insertion points, every old id u moves to u + (new keys at or before it),
// the other lists' ids are shifted by that prefix count (none at all when no key
// is new), and the changed lists look their ids up.  Removed postings leave
// their keys in the dictionary -- an id without postings changes no join --
// until the next full rebuild.

#include <hipcub/hipcub.hpp>

#include "yrwi_host.h"
#include "yrwi_bitmap.h"

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

// the ids of the concatenated lists -> uid_all, whose list slices start on 128-B
// lines: one workgroup per PAD_CHUNK ids of one list (host-built descriptors)
constexpr int PAD_CHUNK = 4096;
struct PadChunk {
  int64_t src, dst;
  int32_t n, pad;
};
__global__ __launch_bounds__(256) void k_pad_copy(const PadChunk* __restrict__ ch, const uint32_t* __restrict__ src,
                                                  uint32_t* __restrict__ dst) {
  const PadChunk c = ch[blockIdx.x];
  for (int x = threadIdx.x; x < c.n; x += 256) dst[c.dst + x] = src[c.src + x];
}

// Line heads of every list (DList::head): level 1 = the first id of each 32-id
// line, level 2 = every 32nd level-1 head.  k_probe searches the heads of a
// probe tile's range in LDS and then reads one leaf line per key.
struct HeadSeg {
  const uint32_t* uid;
  uint32_t* head;
  int64_t n;
};
__global__ void k_heads(const HeadSeg* __restrict__ segs, const int64_t* __restrict__ hoff, int nseg, int64_t nh) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nh) return;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (hoff[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const HeadSeg S = segs[lo];
  const int64_t g = i - hoff[lo];
  const int64_t c1 = head1_cap(S.n);
  if (g < head1_n(S.n)) S.head[g] = S.uid[g << 5];
  else if (g >= c1 && g - c1 < head2_n(S.n)) S.head[g] = S.uid[(g - c1) << 10];
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

// 72-bit key order: (hi, lo) lexicographic
__device__ __forceinline__ bool key_less(uint64_t ah, uint8_t al, uint64_t bh, uint8_t bl) {
  return ah < bh || (ah == bh && al < bl);
}
__device__ __forceinline__ int64_t dict_lower_bound(const uint64_t* __restrict__ dh, const uint8_t* __restrict__ dl,
                                                    int64_t n, uint64_t h, uint8_t l) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (key_less(dh[mid], dl[mid], h, l)) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// distinct sorted keys: key j (a run start) -> slot rank1[j] - 1
__global__ void k_cand_compact(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ rank1,
                               const uint64_t* __restrict__ kh, const uint8_t* __restrict__ kl,
                               const uint32_t* __restrict__ pos, int64_t n, uint64_t* __restrict__ ch,
                               uint8_t* __restrict__ cl) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || !flag[j]) return;
  ch[rank1[j] - 1u] = kh[j];
  cl[rank1[j] - 1u] = kl[pos[j]];
}

// candidate key -> insertion point in the dictionary, and whether it is new
__global__ void k_dict_lookup(const uint64_t* __restrict__ ch, const uint8_t* __restrict__ cl, int64_t nc,
                              const uint64_t* __restrict__ dh, const uint8_t* __restrict__ dl, int64_t nd,
                              uint32_t* __restrict__ ins, uint32_t* __restrict__ isnew) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  const int64_t p = dict_lower_bound(dh, dl, nd, ch[c], cl[c]);
  ins[c] = (uint32_t)p;
  isnew[c] = (p < nd && dh[p] == ch[c] && dl[p] == cl[c]) ? 0u : 1u;
}

// the new keys in order, their insertion points counted per old id
__global__ void k_new_compact(const uint32_t* __restrict__ isnew, const uint32_t* __restrict__ rnew,
                              const uint64_t* __restrict__ ch, const uint8_t* __restrict__ cl,
                              const uint32_t* __restrict__ ins, int64_t nc, uint64_t* __restrict__ nh,
                              uint8_t* __restrict__ nl, uint32_t* __restrict__ nins, uint32_t* __restrict__ hist) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc || !isnew[c]) return;
  const uint32_t j = rnew[c] - 1u;
  nh[j] = ch[c];
  nl[j] = cl[c];
  nins[j] = ins[c];
  atomicAdd(&hist[ins[c]], 1u);
}

// old id u -> u + delta[u] (delta: new keys inserted at or before u)
__global__ void k_dict_move_old(const uint64_t* __restrict__ dh, const uint8_t* __restrict__ dl,
                                const uint32_t* __restrict__ delta, int64_t nd, uint64_t* __restrict__ dh2,
                                uint8_t* __restrict__ dl2) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nd) return;
  dh2[u + delta[u]] = dh[u];
  dl2[u + delta[u]] = dl[u];
}
// new key j lands after ins[j] old keys and j new ones
__global__ void k_dict_put_new(const uint64_t* __restrict__ nh, const uint8_t* __restrict__ nl,
                               const uint32_t* __restrict__ nins, int64_t nn, uint64_t* __restrict__ dh2,
                               uint8_t* __restrict__ dl2) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nn) return;
  dh2[nins[j] + j] = nh[j];
  dl2[nins[j] + j] = nl[j];
}

struct UidSeg {
  uint32_t* uid;
  const uint64_t* khi;
  const uint8_t* klo;
};
__device__ __forceinline__ int seg_of(const int64_t* __restrict__ off, int nseg, int64_t i) {
  int lo = 0, hi = nseg - 1;  // last segment with off <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}
// unchanged lists: ids shift by the new keys before them
__global__ void k_uid_remap(const UidSeg* __restrict__ segs, const int64_t* __restrict__ off, int nseg, int64_t n,
                            const uint32_t* __restrict__ delta) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = seg_of(off, nseg, i);
  uint32_t* u = segs[s].uid + (i - off[s]);
  *u += delta[*u];
}
// changed lists: ids looked up in the (updated) dictionary
__global__ void k_uid_assign(const UidSeg* __restrict__ segs, const int64_t* __restrict__ off, int nseg, int64_t n,
                             const uint64_t* __restrict__ dh, const uint8_t* __restrict__ dl, int64_t nd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = seg_of(off, nseg, i);
  const int64_t j = i - off[s];
  segs[s].uid[j] = (uint32_t)dict_lower_bound(dh, dl, nd, segs[s].khi[j], segs[s].klo[j]);
}
// consistency: every posting's id names its key, ids ascend within a list, the dictionary ascends
__global__ void k_uid_check(const UidSeg* __restrict__ segs, const int64_t* __restrict__ off, int nseg, int64_t n,
                            const uint64_t* __restrict__ dh, const uint8_t* __restrict__ dl, int64_t nd,
                            unsigned long long* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nd && i > 0 && !key_less(dh[i - 1], dl[i - 1], dh[i], dl[i])) atomicAdd(bad, 1ull);
  if (i >= n) return;
  const int s = seg_of(off, nseg, i);
  const int64_t j = i - off[s];
  const uint32_t u = segs[s].uid[j];
  bool ok = (int64_t)u < nd && dh[u] == segs[s].khi[j] && dl[u] == segs[s].klo[j];
  if (ok && j > 0) ok = segs[s].uid[j - 1] < u;
  if (!ok) atomicAdd(bad, 1ull);
}

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

// url-id bitmaps of the large lists (DList::bm, yrwi_bitmap.h): per posting, its
// id's bit, and the list position of the first posting of every 96-id unit (its rank)
struct BmSeg {
  const uint32_t* uid;
  uint64_t* bm;
  int64_t n;
  const uint64_t* feat;  // the list's records, and
  uint64_t* j5;          // their words 0-1 (DList::j5), nullptr: none
};
__global__ void k_bitmap_set(const BmSeg* __restrict__ segs, const int64_t* __restrict__ off, int nseg, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const BmSeg S = segs[lo];
  const int64_t j = i - off[lo];
  const uint32_t u = S.uid[j];
  const BmAt a = bm_at(u);
  uint32_t* b32 = reinterpret_cast<uint32_t*>(S.bm) + (size_t)a.unit * 4;
  atomicOr(b32 + (a.bit >> 5), 1u << (a.bit & 31u));
  if (j == 0 || bm_at(S.uid[j - 1]).unit != a.unit) b32[3] = (uint32_t)j;  // the unit's first posting
  if (S.j5) reinterpret_cast<ulonglong2*>(S.j5)[j] = reinterpret_cast<const ulonglong2*>(S.feat + j * FEAT_WORDS)[0];
}

// bitmap lists: every posting's bit is set and its unit's rank + the bits below give its position
__global__ void k_bitmap_check(const BmSeg* __restrict__ segs, const int64_t* __restrict__ off, int nseg, int64_t n,
                               unsigned long long* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const BmSeg S = segs[lo];
  const int64_t j = i - off[lo];
  const uint32_t u = S.uid[j];
  const BmAt a = bm_at(u);
  const uint4 U = reinterpret_cast<const uint4*>(S.bm)[a.unit];
  if (!bm_test(a, U) || bm_pos(a, U) != j) atomicAdd(bad, 1ull);
  if (S.j5 && (S.j5[2 * j] != S.feat[j * FEAT_WORDS] || S.j5[2 * j + 1] != S.feat[j * FEAT_WORDS + 1]))
    atomicAdd(bad, 1ull);
}

__global__ void k_heads_check(const HeadSeg* __restrict__ segs, const int64_t* __restrict__ hoff, int nseg,
                              int64_t nh, unsigned long long* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nh) return;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (hoff[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const HeadSeg S = segs[lo];
  const int64_t g = i - hoff[lo];
  const int64_t c1 = head1_cap(S.n);
  if (S.head == nullptr) {
    if (g == 0) atomicAdd(bad, 1ull);
  } else if (g < head1_n(S.n)) {
    if (S.head[g] != S.uid[g << 5]) atomicAdd(bad, 1ull);
  } else if (g >= c1 && g - c1 < head2_n(S.n)) {
    if (S.head[g] != S.uid[(g - c1) << 10]) atomicAdd(bad, 1ull);
  }
}

}  // namespace

namespace {

// keys of the postings of `lists`, sorted (klo, then stably khi), with run flags
// and ranks: sorted key j = (kh[j], kl[pos[j]]), rank1[j] = 1 + its distinct rank
struct SortedKeys {
  DevBuf bsegs, boff, bkh, bkh2, bkl, bkl2, bpos, bpos2, bflag, brank, btmp;
  uint64_t* kh = nullptr;
  uint8_t* kl = nullptr;
  uint32_t *pos = nullptr, *flag = nullptr, *rank1 = nullptr;
  int64_t n = 0;
  uint32_t ndistinct = 0;
  int nseg = 0;
  const int64_t* d_off = nullptr;  // first posting of every list (concatenation order)
};

int sort_keys(CtxBase* ctx, const std::vector<ListRec*>& lists, SortedKeys& K) {
  hipStream_t st = ctx->stream;
  std::vector<DictSeg> segs;
  std::vector<int64_t> off;
  int64_t n = 0;
  for (ListRec* L : lists) {
    segs.push_back({L->khi, L->klo});
    off.push_back(n);
    n += L->n;
  }
  K.n = n;
  K.nseg = (int)segs.size();
  DictSeg* d_segs = K.bsegs.get<DictSeg>(segs.size());
  int64_t* d_off = K.boff.get<int64_t>(off.size());
  uint64_t* kh = K.bkh.get<uint64_t>((size_t)n);
  uint64_t* kh2 = K.bkh2.get<uint64_t>((size_t)n);
  uint8_t* kl = K.bkl.get<uint8_t>((size_t)n);
  uint8_t* kl2 = K.bkl2.get<uint8_t>((size_t)n);
  uint32_t* pos = K.bpos.get<uint32_t>((size_t)n);
  uint32_t* pos2 = K.bpos2.get<uint32_t>((size_t)n);
  uint32_t* flag = K.bflag.get<uint32_t>((size_t)n);
  uint32_t* rank1 = K.brank.get<uint32_t>((size_t)n);
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
  void* tmp = K.btmp.get<uint8_t>(tb);
  if (!tmp) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
  // (klo) then, stably, (khi): sorted by the 72-bit key; pos = posting index
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t1, kl, kl2, pos, pos2, ni, 0, 8, st));
  hipLaunchKernelGGL(k_gather_u64, dim3(nb(n)), dim3(256), 0, st, kh, pos2, n, kh2);
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t2, kh2, kh, pos2, pos, ni, 0, 64, st));
  hipLaunchKernelGGL(k_dict_flags, dim3(nb(n)), dim3(256), 0, st, kh, pos, kl, n, flag);
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(tmp, t3, flag, rank1, ni, st));
  HIPCHK(ctx, hipMemcpyAsync(&K.ndistinct, rank1 + (n - 1), 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  K.d_off = d_off;
  K.kh = kh;
  K.kl = kl;
  K.pos = pos;
  K.flag = flag;
  K.rank1 = rank1;
  return 0;
}

void publish_dict(CtxBase* ctx) {
  for (Lane* L : ctx->lanes) {  // no batch is in flight while the dictionary changes
    L->dkhi = ctx->dkhi;
    L->dklo = ctx->dklo;
    L->nurls = ctx->nurls;
  }
}

int full_rebuild(CtxBase* ctx, const std::vector<ListRec*>& lists, int64_t n) {
  hipStream_t st = ctx->stream;
  std::vector<int64_t> poff;
  int64_t np = 0;
  for (ListRec* L : lists) {
    poff.push_back(np);
    np += (L->n + 31) & ~(int64_t)31;  // slices start on 128-B lines
  }
  if (np > 0 && (size_t)np > ctx->uid_cap) {
    if (ctx->uid_all) hipFree(ctx->uid_all);
    ctx->uid_all = nullptr;
    ctx->uid_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->uid_all), (size_t)np * 4) != hipSuccess)
      return ctx->fail(YRWI_E_NOMEM, "url id allocation");
    ctx->uid_cap = (size_t)np;
  }
  for (size_t s = 0; s < lists.size(); s++) lists[s]->uid = ctx->uid_all + poff[s];
  SortedKeys K;
  if (int rc = sort_keys(ctx, lists, K)) return rc;
  // ids in concatenation order, then copied into the line-aligned slices
  std::vector<PadChunk> chunks;
  int64_t o = 0;
  for (size_t s = 0; s < lists.size(); s++) {
    for (int64_t x = 0; x < lists[s]->n; x += PAD_CHUNK)
      chunks.push_back({o + x, poff[s] + x, (int32_t)std::min<int64_t>(PAD_CHUNK, lists[s]->n - x), 0});
    o += lists[s]->n;
  }
  DevBuf btmp, bch;
  uint32_t* d_tmp = btmp.get<uint32_t>((size_t)n);
  PadChunk* d_ch = bch.get<PadChunk>(chunks.size());
  if (!d_tmp || !d_ch) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
  HIPCHK(ctx, hipMemcpyAsync(d_ch, chunks.data(), chunks.size() * sizeof(PadChunk), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_dict_scatter, dim3(nb(n)), dim3(256), 0, st, K.rank1, K.pos, n, d_tmp);
  if (!chunks.empty())
    hipLaunchKernelGGL(k_pad_copy, dim3((unsigned)chunks.size()), dim3(256), 0, st, d_ch, d_tmp, ctx->uid_all);
  const uint32_t nurls = K.ndistinct;
  if ((size_t)nurls > ctx->dict_cap) {
    HIPCHK(ctx, hipStreamSynchronize(st));
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
  publish_dict(ctx);
  hipLaunchKernelGGL(k_dict_keys, dim3(nb(n)), dim3(256), 0, st, K.flag, K.rank1, K.kh, K.kl, K.pos, n, ctx->dkhi,
                     ctx->dklo);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipStreamSynchronize(st));  // scratch is freed on return
  ctx->dict_valid = true;
  ctx->dict_churn = 0;
  return 0;
}

std::vector<UidSeg> uid_segs(const std::vector<ListRec*>& lists, std::vector<int64_t>* off, int64_t* n) {
  std::vector<UidSeg> v;
  *n = 0;
  for (ListRec* L : lists) {
    if (L->n == 0) continue;
    v.push_back({L->uid, L->khi, L->klo});
    off->push_back(*n);
    *n += L->n;
  }
  return v;
}

// the lists of ctx->dict_pending (`changed`) merged into a valid dictionary
int incremental(CtxBase* ctx, const std::vector<ListRec*>& changed, const std::vector<ListRec*>& others) {
  hipStream_t st = ctx->stream;
  SortedKeys K;
  if (int rc = sort_keys(ctx, changed, K)) return rc;
  const int64_t nc = K.ndistinct, nd = ctx->nurls;
  DevBuf bch, bcl, bins, bisnew, brnew, btmp;
  uint64_t* ch = bch.get<uint64_t>((size_t)nc);
  uint8_t* cl = bcl.get<uint8_t>((size_t)nc);
  uint32_t* ins = bins.get<uint32_t>((size_t)nc);
  uint32_t* isnew = bisnew.get<uint32_t>((size_t)nc);
  uint32_t* rnew = brnew.get<uint32_t>((size_t)nc);
  if (!ch || !cl || !ins || !isnew || !rnew) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
  hipLaunchKernelGGL(k_cand_compact, dim3(nb(K.n)), dim3(256), 0, st, K.flag, K.rank1, K.kh, K.kl, K.pos, K.n, ch, cl);
  hipLaunchKernelGGL(k_dict_lookup, dim3(nb(nc)), dim3(256), 0, st, ch, cl, nc, ctx->dkhi, ctx->dklo, nd, ins, isnew);
  size_t t1 = 0;
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(nullptr, t1, isnew, rnew, (int)nc, st));
  void* tmp = btmp.get<uint8_t>(std::max<size_t>(t1, 1));
  if (!tmp) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(tmp, t1, isnew, rnew, (int)nc, st));
  uint32_t nn = 0;
  HIPCHK(ctx, hipMemcpyAsync(&nn, rnew + (nc - 1), 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  if (nd + (int64_t)nn > (int64_t)UINT32_MAX) return ctx->fail(YRWI_E_LIMIT, "more than 2^32 urls in one context");
  if (nn > 0) {
    DevBuf bnh, bnl, bnins, bhist, bdelta, btmp2;
    uint64_t* nh = bnh.get<uint64_t>(nn);
    uint8_t* nl = bnl.get<uint8_t>(nn);
    uint32_t* nins = bnins.get<uint32_t>(nn);
    uint32_t* hist = bhist.get<uint32_t>((size_t)nd + 1);
    uint32_t* delta = bdelta.get<uint32_t>((size_t)nd + 1);
    if (!nh || !nl || !nins || !hist || !delta) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
    HIPCHK(ctx, hipMemsetAsync(hist, 0, ((size_t)nd + 1) * 4, st));
    hipLaunchKernelGGL(k_new_compact, dim3(nb(nc)), dim3(256), 0, st, isnew, rnew, ch, cl, ins, nc, nh, nl, nins, hist);
    size_t t2 = 0;
    HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(nullptr, t2, hist, delta, (int)nd + 1, st));
    void* tmp2 = btmp2.get<uint8_t>(std::max<size_t>(t2, 1));
    if (!tmp2) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
    HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(tmp2, t2, hist, delta, (int)nd + 1, st));
    // the grown dictionary (new arrays: old ids move)
    const int64_t nd2 = nd + nn;
    const size_t cap2 = std::max<size_t>((size_t)nd2, ctx->dict_cap);
    uint64_t* dh2 = nullptr;
    uint8_t* dl2 = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&dh2), cap2 * 8) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&dl2), cap2) != hipSuccess) {
      if (dh2) hipFree(dh2);
      return ctx->fail(YRWI_E_NOMEM, "url dictionary allocation");
    }
    hipLaunchKernelGGL(k_dict_move_old, dim3(nb(nd)), dim3(256), 0, st, ctx->dkhi, ctx->dklo, delta, nd, dh2, dl2);
    hipLaunchKernelGGL(k_dict_put_new, dim3(nb(nn)), dim3(256), 0, st, nh, nl, nins, (int64_t)nn, dh2, dl2);
    // every unchanged list's ids shift by the new keys before them
    std::vector<int64_t> off;
    int64_t no = 0;
    std::vector<UidSeg> segs = uid_segs(others, &off, &no);
    DevBuf bsegs, boff;
    if (no > 0) {
      UidSeg* d_segs = bsegs.get<UidSeg>(segs.size());
      int64_t* d_off = boff.get<int64_t>(off.size());
      if (!d_segs || !d_off) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
      HIPCHK(ctx, hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(UidSeg), hipMemcpyHostToDevice, st));
      HIPCHK(ctx, hipMemcpyAsync(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_uid_remap, dim3(nb(no)), dim3(256), 0, st, d_segs, d_off, (int)segs.size(), no, delta);
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipStreamSynchronize(st));
    hipFree(ctx->dkhi);
    hipFree(ctx->dklo);
    ctx->dkhi = dh2;
    ctx->dklo = dl2;
    ctx->dict_cap = cap2;
    ctx->nurls = nd2;
    publish_dict(ctx);
  }
  // the changed lists' ids, looked up in the dictionary
  for (ListRec* L : changed) {
    L->uid = reinterpret_cast<uint32_t*>(ctx->index_mem.alloc((size_t)L->n * 4));
    if (!L->uid) return ctx->fail(YRWI_E_NOMEM, "url id allocation");
  }
  std::vector<int64_t> off;
  int64_t np = 0;
  std::vector<UidSeg> segs = uid_segs(changed, &off, &np);
  DevBuf bsegs, boff;
  UidSeg* d_segs = bsegs.get<UidSeg>(segs.size());
  int64_t* d_off = boff.get<int64_t>(off.size());
  if (!d_segs || !d_off) return ctx->fail(YRWI_E_NOMEM, "url dictionary scratch");
  HIPCHK(ctx, hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(UidSeg), hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_uid_assign, dim3(nb(np)), dim3(256), 0, st, d_segs, d_off, (int)segs.size(), np, ctx->dkhi,
                     ctx->dklo, ctx->nurls);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipStreamSynchronize(st));
  return 0;
}

// every list's line heads, after its url ids changed (all of them shift on an
// incremental update that adds keys): one pass of n/32 + n/1024 id reads
int build_heads(CtxBase* ctx, const std::vector<ListRec*>& lists) {
  hipStream_t st = ctx->stream;
  std::vector<HeadSeg> segs;
  std::vector<int64_t> hoff;
  int64_t nh = 0;
  for (ListRec* L : lists) {
    hoff.push_back(nh);
    nh += heads_cap(L->n);
  }
  if (nh == 0) return 0;
  if ((size_t)nh > ctx->head_cap) {
    if (ctx->head_all) hipFree(ctx->head_all);
    ctx->head_all = nullptr;
    ctx->head_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->head_all), (size_t)nh * 4) != hipSuccess)
      return ctx->fail(YRWI_E_NOMEM, "line head allocation");
    ctx->head_cap = (size_t)nh;
  }
  for (size_t s = 0; s < lists.size(); s++) {
    lists[s]->head = ctx->head_all + hoff[s];
    segs.push_back({lists[s]->uid, lists[s]->head, lists[s]->n});
  }
  DevBuf bsegs, boff;
  HeadSeg* d_segs = bsegs.get<HeadSeg>(segs.size());
  int64_t* d_off = boff.get<int64_t>(hoff.size());
  if (!d_segs || !d_off) return ctx->fail(YRWI_E_NOMEM, "line head scratch");
  HIPCHK(ctx, hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(HeadSeg), hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(d_off, hoff.data(), hoff.size() * 8, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_heads, dim3(nb(nh)), dim3(256), 0, st, d_segs, d_off, (int)segs.size(), nh);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipStreamSynchronize(st));  // scratch is freed on return
  return 0;
}

// Bitmaps for the lists holding at least 1/YRWI_BM_DIV (default 256) of the url
// ids (and 4096 postings): nurls/6 bytes each, so at most 43x the list's own ids
// (at 1/256 density); total capped by YRWI_BM_GB (default 8), largest lists first.
// YRWI_BM_DIV=0: none.  The joins probe only the dense ones (>= 1/64, layout_jobs);
// the sparser ones answer k_chain's tests of a chained fold's later lists and the
// url selections (one word per match instead of a search of the list).
// The dense lists, largest first, get DList::j5 (16 B per posting; total capped by
// YRWI_J5_GB, default 16, apart from the bitmaps' cap; YRWI_J5=0: none): where an
// enumeration's matches sit a few postings apart.
int build_bitmaps(CtxBase* ctx, const std::vector<ListRec*>& lists) {
  hipStream_t st = ctx->stream;
  for (ListRec* L : lists) L->bm = L->j5 = nullptr;
  const char* ej = getenv("YRWI_J5");
  const char* gj = getenv("YRWI_J5_GB");
  const int64_t j5_cap = (ej && atoi(ej) == 0) ? 0 : (int64_t)((gj ? atof(gj) : 16.0) * (double)(1ll << 30));
  const char* e = getenv("YRWI_BM_DIV");
  const int64_t div = e ? atoll(e) : 256;
  const char* g = getenv("YRWI_BM_GB");
  const int64_t cap_bytes = (int64_t)((g ? atof(g) : 8.0) * (double)(1ll << 30));
  if (div <= 0 || ctx->nurls <= 0) return 0;
  const int64_t per = 2 * bm_units(ctx->nurls);  // uint64 per bitmap
  const int64_t thr = std::max<int64_t>(4096, ctx->nurls / div);
  std::vector<ListRec*> big;
  for (ListRec* L : lists)
    if (L->n >= thr) big.push_back(L);
  std::sort(big.begin(), big.end(), [](const ListRec* a, const ListRec* b) { return a->n > b->n; });
  while (!big.empty() && (int64_t)big.size() * per * 8 > cap_bytes) big.pop_back();  // the largest lists first
  if (big.empty()) return 0;
  size_t nj5 = 0;  // lists with a J5 array (the first nj5 of big)
  int64_t j5_words = 0;
  // (the dense lists only, >= 1/64 of the url ids: where an enumeration's matches sit a few postings apart)
  while (nj5 < big.size() && big[nj5]->n * 64 >= ctx->nurls && (j5_words + 2 * big[nj5]->n) * 8 <= j5_cap)
    j5_words += 2 * big[nj5++]->n;
  const size_t bm_words = big.size() * (size_t)per;
  size_t need = bm_words + (size_t)j5_words;
  if (need > ctx->bm_cap) {
    if (ctx->bm_all) hipFree(ctx->bm_all);
    ctx->bm_all = nullptr;
    ctx->bm_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->bm_all), need * 8) != hipSuccess) {
      // the J5 arrays are an optimisation of the compaction, the bitmaps replace
      // whole searches: without room for both, drop the J5 arrays first
      (void)hipGetLastError();
      nj5 = 0;
      j5_words = 0;
      need = bm_words;
      if (hipMalloc(reinterpret_cast<void**>(&ctx->bm_all), need * 8) != hipSuccess) {
        (void)hipGetLastError();
        ctx->bm_all = nullptr;
        return 0;  // no bitmaps: the joins search the lists instead
      }
      fprintf(stderr, "[yrwi] url-id bitmaps without J5 arrays: no device memory for both\n");
    }
    ctx->bm_cap = need;
  }
  HIPCHK(ctx, hipMemsetAsync(ctx->bm_all, 0, bm_words * 8, st));  // the J5 arrays are written whole
  std::vector<BmSeg> segs;
  std::vector<int64_t> off;
  int64_t n = 0, jw = 0;
  for (size_t k = 0; k < big.size(); k++) {
    big[k]->bm = ctx->bm_all + k * (size_t)per;
    if (k < nj5) {
      big[k]->j5 = ctx->bm_all + bm_words + (size_t)jw;
      jw += 2 * big[k]->n;
    }
    segs.push_back({big[k]->uid, big[k]->bm, big[k]->n, big[k]->feat, big[k]->j5});
    off.push_back(n);
    n += big[k]->n;
  }
  DevBuf bsegs, boff;
  BmSeg* d_segs = bsegs.get<BmSeg>(segs.size());
  int64_t* d_off = boff.get<int64_t>(off.size());
  if (!d_segs || !d_off) return ctx->fail(YRWI_E_NOMEM, "bitmap scratch");
  HIPCHK(ctx, hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(BmSeg), hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_bitmap_set, dim3(nb(n)), dim3(256), 0, st, d_segs, d_off, (int)segs.size(), n);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipStreamSynchronize(st));
  return 0;
}

// Index memory is a bump arena: a replaced or removed list's rows, keys, records
// and (incrementally assigned) url ids stay allocated.  Once the dead bytes pass
// the live ones (and 256 MB), every live list is copied into one fresh chunk and
// the old chunks are freed, so a list re-put again and again (IndexCell.add)
// costs device memory in proportion to its current size, not to its history.
// Url ids inside uid_all (full rebuild) stay where they are.  No batch is in
// flight (callers drain).
static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

int repack_index(CtxBase* ctx, bool force) {
  auto in_uid_all = [&](const ListRec& L) {
    return ctx->uid_all && L.uid >= ctx->uid_all && L.uid < ctx->uid_all + ctx->uid_cap;
  };
  size_t live = 0;
  for (auto& kv : ctx->lists) {
    const ListRec& L = kv.second;
    if (L.n == 0) continue;
    live += al256((size_t)L.n * 40) + al256((size_t)L.n * 8) + al256((size_t)L.n);
    if (L.feat) live += al256((size_t)L.n * FEAT_BYTES);
    if (L.uid && !in_uid_all(L)) live += al256((size_t)L.n * 4);
  }
  const size_t used = ctx->index_mem.total_used;
  const size_t dead = used > live ? used - live : 0;
  const char* e = getenv("YRWI_REPACK_MIN_MB");  // read per call: tests lower it
  const size_t min_dead = (size_t)((e ? atof(e) : 256.0) * (double)(1 << 20));
  if (!force && (dead <= live || dead < min_dead)) return 0;
  // a repack that failed for want of memory is not retried until the index changes
  if (!force && ctx->repack_blocked_at == used) return 0;
  hipStream_t st = ctx->stream;
  // Transactional: every live list is copied into `fresh` while its new pointers
  // collect in a side table; they replace the lists' pointers only once every copy
  // is enqueued.  On failure `fresh` is freed and the old layout stays in use.
  Arena fresh(ctx->index_mem.min_chunk);
  if (live > 0) fresh.reserve(live);
  auto move = [&](auto*& ptr, size_t bytes) -> bool {
    using T = std::remove_reference_t<decltype(*ptr)>;
    if (!ptr || bytes == 0) return true;
    uint8_t* q = fresh.alloc(bytes);
    if (!q) return false;
    if (hipMemcpyAsync(q, ptr, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess) return false;
    ptr = reinterpret_cast<T*>(q);
    return true;
  };
  std::vector<std::pair<ListRec*, ListRec>> moved;
  moved.reserve(ctx->lists.size());
  bool ok = true;
  for (auto& kv : ctx->lists) {
    ListRec& L = kv.second;
    if (L.n == 0) continue;
    const size_t n = (size_t)L.n;
    ListRec N = L;
    ok = move(N.rows, n * 40) && move(N.khi, n * 8) && move(N.klo, n) &&
         (N.feat ? move(N.feat, n * FEAT_BYTES) : true) && (N.uid && !in_uid_all(N) ? move(N.uid, n * 4) : true);
    if (!ok) break;
    moved.emplace_back(&L, N);
  }
  if (!ok) {
    hipStreamSynchronize(st);  // copies into `fresh` may be in flight
    fresh.release();
    ctx->repack_blocked_at = used;
    fprintf(stderr, "[yrwi] index repack skipped: no device memory for %.1f MB of live lists (old layout kept)\n",
            live / 1e6);
    return 0;
  }
  for (auto& m : moved) *m.first = m.second;
  HIPCHK(ctx, hipStreamSynchronize(st));
  ctx->index_mem.release();
  ctx->index_mem.chunks.swap(fresh.chunks);
  ctx->index_mem.used = fresh.used;
  ctx->index_mem.cur = fresh.cur;
  ctx->index_mem.total_used = fresh.total_used;
  ctx->index_repacks++;
  // the line heads and bitmaps point at url ids that may have moved: rebuilt next
  ctx->uid_dirty = true;
  return 0;
}

// ------------------------------------------------------------ dense host ids
// Authority (ReferenceOrder.java:176-216) counts the joined postings per host.
// Every url id's host hash (its key's low 36 bits) gets a dense id (the rank of
// the host among the context's distinct hosts), and every index record carries
// its url's id in word 3 (bits 34..63): the host counts then key on a field of
// the record the ranking kernels already read, instead of gathering each
// posting's url key from the dictionary (two random lines per posting).
__global__ void k_host_keys(const uint64_t* __restrict__ dh, const uint8_t* __restrict__ dl, int64_t n,
                            uint64_t* __restrict__ hk, uint32_t* __restrict__ idx) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  hk[u] = ((dh[u] & 0xFFFFFFFull) << 8) | (uint64_t)dl[u];
  idx[u] = (uint32_t)u;
}
__global__ void k_host_flags(const uint64_t* __restrict__ hk, int64_t n, uint32_t* __restrict__ flag) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) flag[j] = (j == 0 || hk[j] != hk[j - 1]) ? 1u : 0u;
}
__global__ void k_host_scatter(const uint64_t* __restrict__ hk, const uint32_t* __restrict__ idx,
                               const uint32_t* __restrict__ flag, const uint32_t* __restrict__ rank1, int64_t n,
                               uint32_t* __restrict__ hid, uint64_t* __restrict__ host_key) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t h = rank1[j] - 1u;
  hid[idx[j]] = h;
  if (flag[j]) host_key[h] = hk[j];
}
struct StampSeg {
  const uint32_t* uid;
  uint64_t* feat;
};
__global__ void k_host_stamp(const StampSeg* __restrict__ segs, const int64_t* __restrict__ off, int nseg, int64_t n,
                             const uint32_t* __restrict__ hid) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = seg_of(off, nseg, i);
  const int64_t j = i - off[s];
  uint64_t* w3 = segs[s].feat + j * FEAT_WORDS + 3;
  *w3 = (*w3 & 0x3FFFFFFFFull) | (uint64_t)hid[segs[s].uid[j]] << 34;
}

}  // namespace

int ensure_host_ids(CtxBase* ctx) {
  if (ctx->host_ids || ctx->uid_dirty || ctx->nurls <= 0) return 0;
  hipStream_t st = ctx->stream;
  const int64_t n = ctx->nurls;
  if (n > (int64_t)INT32_MAX) return 0;  // (the key path serves)
  DevBuf bhk, bhk2, bidx, bidx2, bflag, brank, bhid, btmp;
  uint64_t* hk = bhk.get<uint64_t>((size_t)n);
  uint64_t* hk2 = bhk2.get<uint64_t>((size_t)n);
  uint32_t* idx = bidx.get<uint32_t>((size_t)n);
  uint32_t* idx2 = bidx2.get<uint32_t>((size_t)n);
  uint32_t* flag = bflag.get<uint32_t>((size_t)n);
  uint32_t* rank1 = brank.get<uint32_t>((size_t)n);
  uint32_t* hid = bhid.get<uint32_t>((size_t)n);
  if (!hk || !hk2 || !idx || !idx2 || !flag || !rank1 || !hid) return ctx->fail(YRWI_E_NOMEM, "host id scratch");
  hipLaunchKernelGGL(k_host_keys, dim3(nb(n)), dim3(256), 0, st, ctx->dkhi, ctx->dklo, n, hk, idx);
  size_t t1 = 0, t2 = 0;
  const int ni = (int)n;
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t1, hk, hk2, idx, idx2, ni, 0, 36, st));
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(nullptr, t2, flag, rank1, ni, st));
  void* tmp = btmp.get<uint8_t>(std::max(t1, t2));
  if (!tmp) return ctx->fail(YRWI_E_NOMEM, "host id scratch");
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t1, hk, hk2, idx, idx2, ni, 0, 36, st));
  hipLaunchKernelGGL(k_host_flags, dim3(nb(n)), dim3(256), 0, st, hk2, n, flag);
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(tmp, t2, flag, rank1, ni, st));
  uint32_t nh = 0;
  HIPCHK(ctx, hipMemcpyAsync(&nh, rank1 + (n - 1), 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  if (nh >= (1u << 30)) return 0;  // ids must fit the record's 30 bits (the key path serves)
  if ((size_t)nh > ctx->host_key_cap) {
    if (ctx->host_key) hipFree(ctx->host_key);
    ctx->host_key = nullptr;
    ctx->host_key_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->host_key), (size_t)nh * 8) != hipSuccess)
      return ctx->fail(YRWI_E_NOMEM, "host key table");
    ctx->host_key_cap = nh;
  }
  hipLaunchKernelGGL(k_host_scatter, dim3(nb(n)), dim3(256), 0, st, hk2, idx2, flag, rank1, n, hid, ctx->host_key);
  std::vector<StampSeg> segs;
  std::vector<int64_t> off;
  int64_t np = 0;
  for (auto& kv : ctx->lists) {
    const ListRec& L = kv.second;
    if (L.n == 0 || !L.feat || !L.uid) continue;
    segs.push_back({L.uid, L.feat});
    off.push_back(np);
    np += L.n;
  }
  DevBuf bsegs, boff;
  if (np > 0) {
    StampSeg* d_segs = bsegs.get<StampSeg>(segs.size());
    int64_t* d_off = boff.get<int64_t>(off.size());
    if (!d_segs || !d_off) return ctx->fail(YRWI_E_NOMEM, "host id scratch");
    HIPCHK(ctx, hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(StampSeg), hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_host_stamp, dim3(nb(np)), dim3(256), 0, st, d_segs, d_off, (int)segs.size(), np, hid);
  }
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipStreamSynchronize(st));  // scratch is freed on return
  ctx->nhosts = nh;
  ctx->host_ids = true;
  for (Lane* L : ctx->lanes) {
    L->host_ids = true;
    L->host_key = ctx->host_key;
  }
  return 0;
}

void index_changed(CtxBase* ctx, const KeyT& term, int64_t old_n, bool added) {
  ctx->uid_dirty = true;
  ctx->host_ids = false;  // a new list's records carry no host ids; new urls may bring new hosts
  for (Lane* L : ctx->lanes) L->host_ids = false;
  ctx->dict_churn += old_n;
  if (added) ctx->dict_pending.insert(term);
  else ctx->dict_pending.erase(term);
}

int ensure_url_ids(CtxBase* ctx) {
  if (!ctx->uid_dirty) return 0;
  if (int rc = repack_index(ctx, false)) return rc;
  hipStream_t st = ctx->stream;
  std::vector<ListRec*> lists, changed, others;
  int64_t n = 0, nchanged = 0;
  for (auto& kv : ctx->lists) {
    if (kv.second.n == 0) continue;
    lists.push_back(&kv.second);
    n += kv.second.n;
    if (ctx->dict_pending.count(kv.first)) {
      changed.push_back(&kv.second);
      nchanged += kv.second.n;
    } else {
      others.push_back(&kv.second);
    }
  }
  if (n > (int64_t)INT32_MAX) return ctx->fail(YRWI_E_LIMIT, "more than 2^31 postings in one context");
  // ranking records of lists that have none yet (new or replaced lists)
  for (ListRec* L : lists) {
    if (L->feat) continue;
    L->feat = reinterpret_cast<uint64_t*>(ctx->index_mem.alloc((size_t)L->n * FEAT_BYTES));
    if (!L->feat) return ctx->fail(YRWI_E_NOMEM, "ranking record allocation");
    if (launch_features(L->rows, L->n, L->feat, st)) return ctx->fail(YRWI_E_HIP, "features launch");
  }
  int rc = 0;
  if (n == 0) {
    ctx->dict_valid = false;
  } else {
    // a full rebuild when there is no dictionary yet, when the changed lists hold a
    // large share of the postings, or when removed postings' keys pile up
    const char* e = getenv("YRWI_DICT_FULL");
    const bool full = !ctx->dict_valid || ctx->nurls == 0 || (e && atoi(e)) || 4 * nchanged > n ||
                      2 * ctx->dict_churn > n;
    rc = full ? full_rebuild(ctx, lists, n) : (changed.empty() ? 0 : incremental(ctx, changed, others));
    if (!rc && full) ctx->dict_full_builds++;
    if (!rc && !full && !changed.empty()) ctx->dict_incremental++;
  }
  if (rc) {
    ctx->dict_valid = false;  // the next call rebuilds in full
    return rc;
  }
  if ((rc = build_heads(ctx, lists)) || (rc = build_bitmaps(ctx, lists))) {
    ctx->dict_valid = false;
    return rc;
  }
  ctx->dict_pending.clear();
  ctx->uid_dirty = false;
  measure_scratch(ctx);  // what the index leaves for the lanes' scratch
  return 0;
}

int check_url_ids(CtxBase* ctx, int64_t* bad) {
  *bad = 0;
  if (int rc = ensure_url_ids(ctx)) return rc;
  hipStream_t st = ctx->stream;
  std::vector<ListRec*> lists;
  for (auto& kv : ctx->lists)
    if (kv.second.n) lists.push_back(&kv.second);
  std::vector<int64_t> off;
  int64_t n = 0;
  std::vector<UidSeg> segs = uid_segs(lists, &off, &n);
  const int64_t m = std::max<int64_t>(n, ctx->nurls);
  if (m == 0) return 0;
  DevBuf bsegs, boff, bbad;
  UidSeg* d_segs = bsegs.get<UidSeg>(std::max<size_t>(segs.size(), 1));
  int64_t* d_off = boff.get<int64_t>(std::max<size_t>(off.size(), 1));
  unsigned long long* d_bad = bbad.get<unsigned long long>(1);
  if (!d_segs || !d_off || !d_bad) return ctx->fail(YRWI_E_NOMEM, "check scratch");
  if (!segs.empty()) {
    HIPCHK(ctx, hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(UidSeg), hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, st));
  }
  HIPCHK(ctx, hipMemsetAsync(d_bad, 0, 8, st));
  hipLaunchKernelGGL(k_uid_check, dim3(nb(m)), dim3(256), 0, st, d_segs, d_off, (int)segs.size(), n, ctx->dkhi,
                     ctx->dklo, ctx->nurls, d_bad);
  // every list's line heads name the ids they copy (k_probe relies on them)
  std::vector<HeadSeg> hsegs;
  std::vector<int64_t> hoff;
  int64_t nh = 0;
  for (ListRec* L : lists) {
    hsegs.push_back({L->uid, L->head, L->n});
    hoff.push_back(nh);
    nh += heads_cap(L->n);
  }
  DevBuf bh, bho;
  if (nh > 0) {
    HeadSeg* d_h = bh.get<HeadSeg>(hsegs.size());
    int64_t* d_ho = bho.get<int64_t>(hoff.size());
    if (!d_h || !d_ho) return ctx->fail(YRWI_E_NOMEM, "check scratch");
    HIPCHK(ctx, hipMemcpyAsync(d_h, hsegs.data(), hsegs.size() * sizeof(HeadSeg), hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(d_ho, hoff.data(), hoff.size() * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_heads_check, dim3(nb(nh)), dim3(256), 0, st, d_h, d_ho, (int)hsegs.size(), nh, d_bad);
  }
  std::vector<BmSeg> vbs;
  std::vector<int64_t> vbo;
  int64_t nbm = 0;
  for (ListRec* L : lists)
    if (L->bm) {
      vbs.push_back({L->uid, L->bm, L->n, L->feat, L->j5});
      vbo.push_back(nbm);
      nbm += L->n;
    }
  DevBuf bb, bbo;
  if (nbm > 0) {
    BmSeg* d_b = bb.get<BmSeg>(vbs.size());
    int64_t* d_bo = bbo.get<int64_t>(vbo.size());
    if (!d_b || !d_bo) return ctx->fail(YRWI_E_NOMEM, "check scratch");
    HIPCHK(ctx, hipMemcpyAsync(d_b, vbs.data(), vbs.size() * sizeof(BmSeg), hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(d_bo, vbo.data(), vbo.size() * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_bitmap_check, dim3(nb(nbm)), dim3(256), 0, st, d_b, d_bo, (int)vbs.size(), nbm, d_bad);
  }
  unsigned long long hb = 0;
  HIPCHK(ctx, hipMemcpyAsync(&hb, d_bad, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  *bad = (int64_t)hb;
  return 0;
}

}  // namespace yrwi
