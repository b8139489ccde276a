// yrwi_kernels.hip -- gfx950 kernels of the YaCy RWI query hot path.
//
//   k_validate   put_list: url-hash keys (Base64Order) + row checks
//   k_partition  merge-path split points of every join tile
//   k_join       sorted-list intersection of ReferenceContainers by url hash
//                (ReferenceContainer.joinConstructive :397-489) or exclusion
//                marking (excludeDestructive :491-571)
//   k_scan_tiles per-job exclusive scan of tile match counts (order preserving)
//   k_compact    joined 40-byte rows (WordReferenceVars.join :465-499 and
//                toRowEntry :301-322 -> WordReferenceRow ctor :116-161)
//   k_reduce     per-chunk normalisation summary (ReferenceOrder.NormalizeWorker
//                :163-210; WordReferenceVars.min/max :383-455)
//   k_shard_fin  per-query, per-shard summary (ordered fold of chunk summaries)
//   k_combine    settled min/max + max-distance fold over shards
//   k_score      ReferenceOrder.cardinal :223-265 + per-chunk top-k in the
//                WeakPriorityBlockingQueue order (:119-134, :414-425)
//   k_topq       per-query top-k over the chunk candidate lists
//   k_emit       yrwi_hit records
//
// Java int/long semantics are reproduced with explicit uint32_t/uint64_t
// arithmetic (wrap-around, shift counts masked with 31).  Built with
// -ffp-contract=off so the one fp64 term (tf) rounds exactly like Java.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "yrwi_internal.h"
#include "yrwi_bitmap.h"

namespace yrwi {

// ------------------------------------------------------------- helpers
__device__ __forceinline__ int ahpla(uint32_t c) {
  if (c >= 'A' && c <= 'Z') return (int)c - 'A';
  if (c >= 'a' && c <= 'z') return (int)c - 'a' + 26;
  if (c >= '0' && c <= '9') return (int)c - '0' + 52;
  if (c == '-') return 62;
  if (c == '_') return 63;
  return -1;
}

__device__ __forceinline__ int32_t add32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
__device__ __forceinline__ int32_t sub32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
__device__ __forceinline__ int32_t mul32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
__device__ __forceinline__ int32_t shl32(int32_t a, int32_t n) { return (int32_t)((uint32_t)a << (n & 31)); }
__device__ __forceinline__ int32_t div32(int32_t a, int32_t b) {
  if (b == -1) return (int32_t)(0u - (uint32_t)a);
  return a / b;
}
__device__ __forceinline__ int64_t add64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__device__ __forceinline__ int32_t d2i(double d) {  // Java (int) cast
  if (d != d) return 0;
  if (d >= 2147483647.0) return 2147483647;
  if (d <= -2147483648.0) return (int32_t)0x80000000u;
  return (int32_t)d;
}

__device__ __forceinline__ int32_t micro_date_days(int64_t ms) { return (int32_t)((ms / DAY_MS) % 262144LL); }
// microDateDays(reverseMicroDateDays(days)) (MicroDate.java:37-55)
__device__ __forceinline__ int32_t clamp_days(int32_t days, int64_t now_ms) {
  int64_t v = (int64_t)((uint64_t)(int64_t)days * (uint64_t)DAY_MS);
  return micro_date_days(v < now_ms ? v : now_ms);
}

struct Row {
  uint64_t w[5];
  __device__ __forceinline__ uint32_t b(int i) const { return (uint32_t)(w[i >> 3] >> (8 * (i & 7))) & 0xFFu; }
  __device__ __forceinline__ uint32_t u16(int i) const { return (b(i) << 8) | b(i + 1); }
  __device__ __forceinline__ void set(int i, uint32_t v) {
    const int s = 8 * (i & 7);
    w[i >> 3] = (w[i >> 3] & ~(0xFFull << s)) | ((uint64_t)(v & 0xFFu) << s);
  }
};

__device__ __forceinline__ Row load_row(const uint8_t* p) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
  Row r;
#pragma unroll
  for (int i = 0; i < 5; i++) r.w[i] = q[i];
  return r;
}
__device__ __forceinline__ void store_row(uint8_t* p, const Row& r) {
  uint64_t* q = reinterpret_cast<uint64_t*>(p);
#pragma unroll
  for (int i = 0; i < 5; i++) q[i] = r.w[i];
}

// row byte offsets (WordReferenceRow.java:49-72)
enum : int {
  O_A = 12, O_S = 14, O_U = 16, O_W = 17, O_P = 19, O_D = 21, O_L = 22, O_X = 24, O_Y = 25,
  O_M = 26, O_N = 27, O_G = 28, O_Z = 29, O_C = 33, O_T = 34, O_R = 36, O_O = 37, O_I = 38, O_K = 39
};

__device__ __forceinline__ bool key_le(uint64_t ah, uint32_t al, uint64_t bh, uint32_t bl) {
  return ah < bh || (ah == bh && al <= bl);
}

template <class T>
__device__ __forceinline__ int find_job(const int64_t* base, int n, T b) {
  int lo = 0, hi = n - 1;  // largest j with base[j] <= b
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (base[mid] <= (int64_t)b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Global (address space 1) accesses through device pointers that reach a kernel
// inside structs (JoinQ, RankQ, LDS copies of them).  Through a generic pointer
// the compiler emits FLAT instructions, which count in lgkmcnt as well as vmcnt:
// every LDS wait after such a load also waited for the memory, so a thread's
// gathers ran one after another (k_score had 483 flat loads, k_compact 60, and a
// vmcnt(0) wait after nearly each).  Every pointer here is device memory.
template <class T>
__device__ __forceinline__ T ldg(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ void stg(T* p, const T& v) {
  *(__attribute__((address_space(1))) T*)p = v;
}
// HIP's vector types are classes: copying one out of an address-space-1 lvalue
// binds its copy constructor's generic reference (a FLAT load again), so the
// 16-byte forms go through clang's native vector types
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x3_t __attribute__((ext_vector_type(3)));
// the J5 inputs of a joined side: word 0 and the low half of word 1 (12 B: a
// 16-B load whose unused top dword the compiler reused made the next gather wait)
__device__ __forceinline__ ulonglong2 ldg_j5(const uint64_t* p) {
  const u32x3_t v = *(const __attribute__((address_space(1))) u32x3_t*)p;
  return make_ulonglong2((uint64_t)v.y << 32 | v.x, (uint64_t)v.z);
}
template <>
__device__ __forceinline__ ulonglong2 ldg(const ulonglong2* p) {
  const u64x2_t v = *(const __attribute__((address_space(1))) u64x2_t*)p;
  return make_ulonglong2(v.x, v.y);
}
template <>
__device__ __forceinline__ uint4 ldg(const uint4* p) {
  const u32x4_t v = *(const __attribute__((address_space(1))) u32x4_t*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <>
__device__ __forceinline__ uint2 ldg(const uint2* p) {
  const u32x2_t v = *(const __attribute__((address_space(1))) u32x2_t*)p;
  return make_uint2(v.x, v.y);
}
template <>
__device__ __forceinline__ void stg(uint2* p, const uint2& v) {
  u32x2_t w;
  w.x = v.x;
  w.y = v.y;
  *(__attribute__((address_space(1))) u32x2_t*)p = w;
}
template <>
__device__ __forceinline__ void stg(ulonglong2* p, const ulonglong2& v) {
  u64x2_t w;
  w.x = v.x;
  w.y = v.y;
  *(__attribute__((address_space(1))) u64x2_t*)p = w;
}

// wave (64-lane) inclusive scan / reductions
__device__ __forceinline__ int32_t wave_incl_sum(int32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}
__device__ __forceinline__ int32_t wave_incl_max(int32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v = max(v, t);
  }
  return v;
}

// block exclusive scan (sum) for 256 threads; returns exclusive prefix, total in *tot
__device__ __forceinline__ int32_t block_excl_sum256(int32_t v, int32_t* sh /*4*/, int32_t* tot) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t inc = wave_incl_sum(v);
  if (lane == 63) sh[wv] = inc;
  __syncthreads();
  int32_t off = 0, all = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i < wv) off += sh[i];
    all += sh[i];
  }
  __syncthreads();
  *tot = all;
  return off + inc - v;
}
// the same for 64-bit sums (packed counters)
__device__ __forceinline__ uint64_t block_excl_sum256_u64(uint64_t v, uint64_t* sh /*4*/, uint64_t* tot) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) sh[wv] = inc;
  __syncthreads();
  uint64_t off = 0, all = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i < wv) off += sh[i];
    all += sh[i];
  }
  __syncthreads();
  *tot = all;
  return off + inc - v;
}
__device__ __forceinline__ int32_t block_excl_max256(int32_t v, int32_t* sh /*4*/) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int32_t inc = wave_incl_max(v);
  int32_t prev = __shfl_up(inc, 1, 64);
  if (lane == 0) prev = -1;
  if (lane == 63) sh[wv] = inc;
  __syncthreads();
  int32_t off = -1;
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (i < wv) off = max(off, sh[i]);
  __syncthreads();
  return max(off, prev);
}

// ============================================================ uploads
// One launch copies every staged range of an upload (yrwi_host.h upload_list):
// COPY_IN_BLOCK bytes per workgroup, 16 B per thread per step, read from pinned
// host memory through its device address.  Ranges start 256-B aligned on both
// sides (stage offsets, arena allocations); a range's tail is copied bytewise.
constexpr int COPY_IN_BLOCK = 16384;
__global__ __launch_bounds__(256) void k_copy_in(CopyIn c) {
  uint32_t b = blockIdx.x;
  int e = 0;
  for (; e < c.n; e++) {
    const uint32_t nb = (uint32_t)((c.bytes[e] + COPY_IN_BLOCK - 1) / COPY_IN_BLOCK);
    if (b < nb) break;
    b -= nb;
  }
  if (e >= c.n) return;
  const uint8_t* __restrict__ src = c.src[e];
  uint8_t* __restrict__ dst = c.dst[e];
  const uint64_t n = c.bytes[e];
  const uint64_t end = min<uint64_t>(n, (uint64_t)(b + 1) * COPY_IN_BLOCK);
  for (uint64_t o = (uint64_t)b * COPY_IN_BLOCK + threadIdx.x * 16u; o < end; o += 256 * 16) {
    if (o + 16 <= end) {
      *reinterpret_cast<uint4*>(dst + o) = *reinterpret_cast<const uint4*>(src + o);
    } else {
      for (uint64_t x = o; x < end; x++) dst[x] = src[x];
    }
  }
}

int launch_copy_in(const CopyIn& c, void* stream) {
  uint32_t blocks = 0;
  for (int e = 0; e < c.n; e++) blocks += (uint32_t)((c.bytes[e] + COPY_IN_BLOCK - 1) / COPY_IN_BLOCK);
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(k_copy_in, dim3(blocks), dim3(256), 0, (hipStream_t)stream, c);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void k_gather_out(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t n, int32_t elem,
                             int64_t stride, int words) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (words) {
    for (int b = 0; b < elem; b += 4)
      *reinterpret_cast<uint32_t*>(dst + i * elem + b) = *reinterpret_cast<const uint32_t*>(src + i * stride + b);
  } else {
    for (int b = 0; b < elem; b++) dst[i * elem + b] = src[i * stride + b];
  }
}

int launch_gather_out(uint8_t* dst, const uint8_t* src, int64_t n, int32_t elem, int64_t stride, void* stream) {
  if (n <= 0) return 0;
  const int words = (elem % 4 == 0 && stride % 4 == 0 && ((uintptr_t)dst % 4) == 0 && ((uintptr_t)src % 4) == 0);
  hipLaunchKernelGGL(k_gather_out, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dst, src, n,
                     elem, stride, words);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ====================================================== put_list validation
// err bits: 1 = malformed hash, 2 = empty language cell, 4 = not strictly ascending
__global__ void k_validate(const uint8_t* __restrict__ rows, int64_t n, uint64_t* __restrict__ khi,
                           uint8_t* __restrict__ klo, int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* r = rows + i * YRWI_ROW_BYTES;
  int bad = 0;
  auto keyof = [&](const uint8_t* h, uint64_t& hi, uint32_t& lo) {
    uint64_t x = 0;
    for (int j = 0; j < 10; j++) {
      int c = ahpla(h[j]);
      bad |= (c < 0);
      x = (x << 6) | (uint64_t)(c & 63);
    }
    int c10 = ahpla(h[10]), c11 = ahpla(h[11]);
    bad |= (c10 < 0) | (c11 < 0);
    hi = (x << 4) | (uint64_t)((c10 & 63) >> 2);
    lo = (uint32_t)(((c10 & 3) << 6) | (c11 & 63));
  };
  uint64_t hi;
  uint32_t lo;
  keyof(r, hi, lo);
  int e = bad ? 1 : 0;
  if (r[O_L] == 0 && r[O_L + 1] == 0) e |= 2;
  if (i > 0) {
    uint64_t ph;
    uint32_t pl;
    keyof(r - YRWI_ROW_BYTES, ph, pl);
    if (!(ph < hi || (ph == hi && pl < lo))) e |= 4;
  }
  khi[i] = hi;
  klo[i] = (uint8_t)lo;
  if (e) atomicOr(err, e);
}

// ==================================================== decoded postings
struct Feat {  // decoded WordReferenceVars fields of one posting
  int32_t f[NF];
  int32_t a, p, od;
  double tf;
  uint32_t z;     // flags (Bitfield bit j = bit j)
  uint32_t lang;  // language cell: byte 22 | byte 23 << 8
  uint32_t d;     // doctype
  int32_t dl;     // DigestURL.domLengthEstimation key: ahpla[urlhash[11]] & 3
};

__device__ __forceinline__ int32_t url_hashcode(const Row& r);

__device__ __forceinline__ Feat decode(const Row& r) {
  Feat x;
  x.f[F_HITCOUNT] = (int32_t)r.b(O_C);
  x.f[F_LLOCAL] = (int32_t)r.b(O_X);
  x.f[F_LOTHER] = (int32_t)r.b(O_Y);
  x.f[F_WORDSINTEXT] = (int32_t)r.u16(O_W);
  x.f[F_PHRASESINTEXT] = (int32_t)r.u16(O_P);
  x.f[F_POSINTEXT] = (int32_t)r.u16(O_T);
  x.f[F_POSINPHRASE] = (int32_t)r.b(O_R);
  x.f[F_POSOFPHRASE] = (int32_t)r.b(O_O);
  x.f[F_URLLENGTH] = (int32_t)r.b(O_M);
  x.f[F_URLCOMPS] = (int32_t)r.b(O_N);
  x.f[F_WORDSINTITLE] = (int32_t)r.b(O_U);
  x.a = (int32_t)r.u16(O_A);
  x.p = x.f[F_POSINTEXT];
  x.od = (int32_t)r.b(O_I);
  // WordReferenceRow.termFrequency (WordReferenceRow.java:355-357)
  x.tf = (double)x.f[F_HITCOUNT] / (double)(x.f[F_WORDSINTEXT] + x.f[F_WORDSINTITLE] + 1);
  x.z = r.b(O_Z) | (r.b(O_Z + 1) << 8) | (r.b(O_Z + 2) << 16) | (r.b(O_Z + 3) << 24);
  x.lang = r.b(O_L) | (r.b(O_L + 1) << 8);
  x.d = r.b(O_D);
  x.dl = ahpla(r.b(11)) & 3;
  return x;
}

// ---- ranking records (FeatRec, yrwi_internal.h)
struct Rec {
  uint64_t w[FEAT_WORDS];
};

__device__ __forceinline__ Rec rec_of_row(const Row& r) {
  Rec q;
  q.w[0] = (uint64_t)r.u16(O_T) | (uint64_t)r.u16(O_W) << 16 | (uint64_t)r.u16(O_P) << 32 | (uint64_t)r.b(O_U) << 48 |
           (uint64_t)r.b(O_C) << 56;
  q.w[1] = (uint64_t)r.b(O_R) | (uint64_t)r.b(O_O) << 8 | (uint64_t)r.b(O_I) << 16 | (uint64_t)r.b(O_X) << 24 |
           (uint64_t)r.b(O_Y) << 32 | (uint64_t)r.b(O_M) << 40 | (uint64_t)r.b(O_N) << 48 | (uint64_t)r.b(O_D) << 56;
  const uint64_t z = r.b(O_Z) | (r.b(O_Z + 1) << 8) | (r.b(O_Z + 2) << 16) | ((uint64_t)r.b(O_Z + 3) << 24);
  q.w[2] = (uint64_t)r.u16(O_A) | (uint64_t)(r.b(O_L) | (r.b(O_L + 1) << 8)) << 16 | z << 32;
  q.w[3] = (uint64_t)(uint32_t)url_hashcode(r) | (uint64_t)(ahpla(r.b(11)) & 3) << 32;
  return q;
}

// record loads: every feat array starts 256-B aligned, records are 32 B
__device__ __forceinline__ Rec load_rec(const uint64_t* f, int64_t e) {
  const ulonglong2* p = reinterpret_cast<const ulonglong2*>(f + e * FEAT_WORDS);
  const ulonglong2 x = ldg(p), y = ldg(p + 1);
  Rec q;
  q.w[0] = x.x;
  q.w[1] = x.y;
  q.w[2] = y.x;
  q.w[3] = y.y;
  return q;
}
__device__ __forceinline__ void store_rec(uint64_t* f, int64_t e, const Rec& q) {
  ulonglong2* p = reinterpret_cast<ulonglong2*>(f + e * FEAT_WORDS);
  stg(p, make_ulonglong2(q.w[0], q.w[1]));
  stg(p + 1, make_ulonglong2(q.w[2], q.w[3]));
}

__device__ __forceinline__ Feat decode_rec(const Rec& q) {
  Feat x;
  const uint64_t w0 = q.w[0], w1 = q.w[1], w2 = q.w[2];
  x.f[F_HITCOUNT] = (int32_t)(w0 >> 56);
  x.f[F_LLOCAL] = (int32_t)((w1 >> 24) & 0xFF);
  x.f[F_LOTHER] = (int32_t)((w1 >> 32) & 0xFF);
  x.f[F_WORDSINTEXT] = (int32_t)((w0 >> 16) & 0xFFFF);
  x.f[F_PHRASESINTEXT] = (int32_t)((w0 >> 32) & 0xFFFF);
  x.f[F_POSINTEXT] = (int32_t)(w0 & 0xFFFF);
  x.f[F_POSINPHRASE] = (int32_t)(w1 & 0xFF);
  x.f[F_POSOFPHRASE] = (int32_t)((w1 >> 8) & 0xFF);
  x.f[F_URLLENGTH] = (int32_t)((w1 >> 40) & 0xFF);
  x.f[F_URLCOMPS] = (int32_t)((w1 >> 48) & 0xFF);
  x.f[F_WORDSINTITLE] = (int32_t)((w0 >> 48) & 0xFF);
  x.a = (int32_t)(w2 & 0xFFFF);
  x.p = x.f[F_POSINTEXT];
  x.od = (int32_t)((w1 >> 16) & 0xFF);
  x.tf = (double)x.f[F_HITCOUNT] / (double)(x.f[F_WORDSINTEXT] + x.f[F_WORDSINTITLE] + 1);
  x.z = (uint32_t)(w2 >> 32);
  x.lang = (uint32_t)((w2 >> 16) & 0xFFFF);
  x.d = (uint32_t)(w1 >> 56);
  x.dl = (int32_t)((q.w[3] >> 32) & 3);
  return x;
}

// 72-bit url-hash key of container element e: its own key, or its url id's in the dictionary
__device__ __forceinline__ void key_at(const RankQ& Q, int64_t e, uint64_t& hi, uint32_t& lo) {
  if (Q.uid) {
    const uint32_t u = ldg(Q.uid + e);
    hi = ldg(Q.dkhi + u);
    lo = ldg(Q.dklo + u);
  } else {
    hi = ldg(Q.ekhi + e);
    lo = ldg(Q.eklo + e);
  }
}
// url-hash chars 6..11 (the host hash, DigestURL :229-296) = the key's low 36 bits
__device__ __forceinline__ uint64_t key_host36(uint64_t hi, uint32_t lo) {
  return ((hi & 0xFFFFFFFull) << 8) | (lo & 0xFFu);
}
// the host of container element e (record q) as the authority host tables key it
// (host_count adds 1): the dense host id its record carries (Q.host_rec, no url
// key gathered), or the host hash of its url key
__device__ __forceinline__ uint64_t elem_host(const RankQ& Q, uint64_t w3, int64_t e) {
  if (Q.host_rec) return w3 >> 34;
  uint64_t hi;
  uint32_t lo;
  key_at(Q, e, hi, lo);
  return key_host36(hi, lo);
}

// =========================================================== join: partition
// One thread per merge tile: the merge-path split of the tile's first and last
// diagonal (two interleaved binary searches on the url-hash keys) -> TileDesc.
__global__ void k_partition(const JoinQ* __restrict__ jobs, const int64_t* __restrict__ tile_base, int njobs,
                            int64_t total_tiles, TileDesc* __restrict__ desc, int64_t* __restrict__ tile_src,
                            uint32_t* __restrict__ tile_key, int32_t* __restrict__ tile_job) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= total_tiles) return;
  const int j = find_job(tile_base, njobs, b);
  const JoinQ& J = jobs[j];
  const int64_t nA = J.A.n, nB = J.B.n;
  const uint32_t* __restrict__ A = J.A.uid;
  const uint32_t* __restrict__ B = J.B.uid;
  const int64_t d0 = (b - tile_base[j]) * JOIN_TILE;
  const int64_t d1 = d0 + JOIN_TILE < nA + nB ? d0 + JOIN_TILE : nA + nB;
  int64_t lo0 = d0 - nB > 0 ? d0 - nB : 0, hi0 = d0 < nA ? d0 : nA;
  int64_t lo1 = d1 - nB > 0 ? d1 - nB : 0, hi1 = d1 < nA ? d1 : nA;
  while (lo0 < hi0 || lo1 < hi1) {
    if (lo0 < hi0) {
      const int64_t mid = (lo0 + hi0) >> 1;
      if (A[mid] <= B[d0 - 1 - mid]) lo0 = mid + 1; else hi0 = mid;
    }
    if (lo1 < hi1) {
      const int64_t mid = (lo1 + hi1) >> 1;
      if (A[mid] <= B[d1 - 1 - mid]) lo1 = mid + 1; else hi1 = mid;
    }
  }
  TileDesc D;
  D.a = A;
  D.b = B;
  D.a0 = lo0;
  D.b0 = d0 - lo0;
  D.na = (int32_t)(lo1 - lo0);
  D.nb = (int32_t)((d1 - lo1) - (d0 - lo0));
  D.nbl = D.nb + ((d1 - lo1) < nB ? 1 : 0);  // + lookahead element B[b1]
  D.job = j;
  D.maxd = J.maxd;
  D.pad = 0;
  desc[b] = D;
  if (tile_src) tile_src[b] = min(D.na, D.nbl);  // matches of the tile <= min(#A, #B + lookahead); k_scan_bounds: its run
  if (tile_job) tile_job[b] = j;
  if (tile_key) {  // url id the tile starts at (k_order_hist / k_order_scatter)
    const uint32_t ka = D.na > 0 ? A[lo0] : 0xFFFFFFFFu, kb = D.nb > 0 ? B[D.b0] : 0xFFFFFFFFu;
    tile_key[b] = min(ka, kb);
  }
}

// joined worddistance (WordReferenceVars.distance :287-294 after join :465-499)
// from the two postings' ranking records (posintext in word 0, stored distance in word 1)
__device__ __forceinline__ int32_t joined_distance(const uint64_t* fa, const uint64_t* fb, int mode) {
  if (mode == JM_TEST_LARGE_B) return (int32_t)((fb[1] >> 16) & 0xFF);
  if (mode == JM_TEST_LARGE_A) return (int32_t)((fa[1] >> 16) & 0xFF);
  const int pa = (int)(fa[0] & 0xFFFF), pb = (int)(fb[0] & 0xFFFF);
  if (pa > 0 && pb > 0) {
    int d = pa > pb ? pa - pb : pb - pa;
    if (d != 0) return d;
  }
  return (int32_t)((fa[1] >> 16) & 0xFF);
}

// ============================================================ join: tiles
constexpr int JOIN_SLOTS = (JOIN_TILE + 1 + JOIN_THREADS - 1) / JOIN_THREADS;  // JOIN_TILE + 1 items max per tile

struct TileKeys {
  uint32_t a[JOIN_SLOTS], b[JOIN_SLOTS];
};

// global (address space 1) pointers: flat loads would also count in lgkmcnt and
// every LDS wait of the merge would then wait for the prefetch as well
typedef __attribute__((address_space(1))) const uint32_t gu32c;

// Tile id loads through two buffer descriptors (A range, B range + lookahead):
// slot x reads A[x] and B[x - na]; the range check returns 0 for the side that
// is out of bounds (or both, past the tile), so the id is the OR of the two and
// there is no per-slot address select.  Descriptor fields are wave-uniform
// (TileDesc arrives through v_readlane).
__device__ __forceinline__ void tile_load(const TileDesc& D, TileKeys& K) {
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(D.a + D.a0), 0, D.na * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(D.b + D.b0), 0, D.nbl * 4, 0x00020000);
#pragma unroll
  for (int s = 0; s < JOIN_SLOTS; s++) {
    const int x = threadIdx.x + s * JOIN_THREADS;
    K.a[s] = __builtin_amdgcn_raw_buffer_load_b32(ra, x * 4, 0, 0);
    K.b[s] = __builtin_amdgcn_raw_buffer_load_b32(rb, (x - D.na) * 4, 0, 0);
  }
}

// Persistent workgroups walk the merge tiles t = blockIdx.x + k*gridDim.x, the
// ids of the next tile loading while the current one is merged out of LDS.
// LDS holds the tile's A ids at [0, na) and B ids (+ lookahead) at [na, na+nbl).
// Each thread finds its 8-item diagonal by binary search, then merges; it keeps
// only two bit masks (took-A, match) and rebuilds the indices of its (rare)
// matches afterwards.
__global__ __launch_bounds__(JOIN_THREADS) void k_join(const JoinQ* __restrict__ jobs,
                                                      const TileDesc* __restrict__ desc, int64_t ntiles,
                                                      uint2* __restrict__ pairs, uint32_t* __restrict__ pair_uid,
                                                      int64_t* __restrict__ tile_src, int32_t* __restrict__ tile_cnt,
                                                      int mark) {
  __shared__ uint32_t sK[JOIN_SLOTS * JOIN_THREADS];
  __shared__ int32_t sScan[4];

  // Tile descriptors travel through VGPRs (lane i holds dword i, read with
  // v_readlane when due): a scalar load would share lgkmcnt with LDS traffic and
  // every LDS wait of the merge would also wait for the next descriptor.
  // lanes TILEDESC_DWORDS and +1 carry the tile's pair run (tile_src)
  const int lane = threadIdx.x & 63;
  auto desc_fetch = [&](int64_t t) -> uint32_t {
    if (t >= ntiles) return 0u;
    if (lane < TILEDESC_DWORDS) return ((const gu32c*)(desc + t))[lane];
    if (!mark && lane < TILEDESC_DWORDS + 2) return ((const gu32c*)(tile_src + t))[lane - TILEDESC_DWORDS];
    return 0u;
  };
  auto desc_get = [&](uint32_t v, int64_t& src) -> TileDesc {
    TileDesc D;
    uint32_t* w = reinterpret_cast<uint32_t*>(&D);
#pragma unroll
    for (int i = 0; i < TILEDESC_DWORDS; i++) w[i] = __builtin_amdgcn_readlane(v, i);
    src = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(v, TILEDESC_DWORDS + 1) << 32) |
                    (uint32_t)__builtin_amdgcn_readlane(v, TILEDESC_DWORDS));
    return D;
  };
  const int64_t G = gridDim.x;
  int64_t b = blockIdx.x;
  if (b >= ntiles) return;
  int64_t srcc;
  TileDesc Dc = desc_get(desc_fetch(b), srcc);
  uint32_t dnext = desc_fetch(b + G);
  TileKeys K;
  tile_load(Dc, K);
  for (; b < ntiles; b += G) {
    const int na = Dc.na, nb = Dc.nb, nbl = Dc.nbl;
#pragma unroll
    for (int s = 0; s < JOIN_SLOTS; s++) sK[threadIdx.x + s * JOIN_THREADS] = K.a[s] | K.b[s];
    __syncthreads();
    // prefetch: ids of the next tile, descriptor of the one after
    const int64_t a0 = Dc.a0, b0 = Dc.b0;
    const int jc = Dc.job, maxd = Dc.maxd;
    const int64_t src = srcc;
    if (b + G < ntiles) {
      Dc = desc_get(dnext, srcc);
      dnext = desc_fetch(b + 2 * G);
      tile_load(Dc, K);
    }
    const uint32_t* sB = sK + na;
    const int dd0 = threadIdx.x * JOIN_IPT;
    const int dtot = na + nb;
    int lo = dd0 - nb > 0 ? dd0 - nb : 0, hi = dd0 < na ? dd0 : na;
    if (dd0 >= dtot) lo = hi = 0;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sK[mid] <= sB[dd0 - 1 - mid]) lo = mid + 1; else hi = mid;
    }
    const int ia0 = lo, ib0 = dd0 - lo;
    int ia = ia0, ib = ib0;
    uint32_t ka = sK[ia], kb = sB[ib];
    uint32_t tbits = 0, mbits = 0;
    const int nstep = dtot - dd0 < JOIN_IPT ? dtot - dd0 : JOIN_IPT;
#pragma unroll
    for (int s = 0; s < JOIN_IPT; s++) {
      if (s < nstep) {
        const bool takeA = ia < na && (ib >= nb || ka <= kb);
        const bool m = takeA && ib < nbl && ka == kb;
        tbits |= (uint32_t)takeA << s;
        mbits |= (uint32_t)m << s;
        ia += takeA;
        ib += !takeA;
        ka = sK[ia];
        kb = sB[ib];
      }
    }
    // index of the A / B element of step s
    auto a_at = [&](int s) { return ia0 + __popc(tbits & ((1u << s) - 1u)); };
    auto b_at = [&](int s) { return ib0 + s - __popc(tbits & ((1u << s) - 1u)); };
    // maxDistance filter (ReferenceContainer.java:442,482; distance <= 65535 always)
    // and exclusion marks need the job's rows; plain joins never touch the job
    if ((mark || maxd < 65535) && __syncthreads_or(mbits != 0)) {
      const JoinQ& J = jobs[jc];
      for (uint32_t m = mbits; m; m &= m - 1) {
        const int st = __ffs(m) - 1;
        if (mark) {
          stg(J.removed + a0 + a_at(st), (uint8_t)1);
        } else {
          const uint64_t* fa = J.A.feat + (a0 + a_at(st)) * FEAT_WORDS;
          const uint64_t* fb = J.B.feat + (b0 + b_at(st)) * FEAT_WORDS;
          if (joined_distance(fa, fb, J.mode) > J.maxd) mbits &= ~(1u << st);
        }
      }
    }
    if (!mark) {
      int32_t tot;
      int32_t off = block_excl_sum256(__popc(mbits), sScan, &tot);
      if (threadIdx.x == 0) tile_cnt[b] = tot;
      if (jobs[jc].count_only) mbits = 0;  // counted only (workgroup-uniform)
      uint2* out = pairs + src;
      uint32_t* outu = pair_uid + src;
      for (uint32_t m = mbits; m; m &= m - 1) {
        const int st = __ffs(m) - 1;
        const int ai = a_at(st);
        out[off] = make_uint2((uint32_t)(a0 + ai), (uint32_t)(b0 + b_at(st)));
        outu[off] = sK[ai];
        off++;
      }
    }
    __syncthreads();  // LDS is rewritten for the next tile
  }
}

// ============================================================ join: probe
// Skewed sizes (the by-test access pattern of joinConstructiveByTest :419-446,
// RowSet.binarySearch RowSet.java:319-335): every small-list key is looked up in
// the large list.  k_probe_part finds, per tile of PROBE_TILE small keys, the
// large-list range that can hold them (two interleaved binary searches per
// thread, all tiles in parallel); k_probe binary-searches each key inside its
// tile's range.  Output and mark semantics are k_join's.

// XCD slices (cdna_hip_programming.md T1): blocks are dealt round-robin over the
// 8 XCDs, so logical block k of XCD x's share maps to slice x of an order; a
// bijection of [0, n) for any n.  (Applied to job order -- consecutive tiles on
// one XCD -- it was measured slower: k_compact 274 -> 465 us, k_probe 201 -> 214 us,
// profiles/archive/r02h_xcd_swizzle.txt; the band orders below use it.)
__device__ __forceinline__ int64_t xcd_slice(int64_t bid, int64_t n) {
  const int64_t q = n >> 3, r = n & 7;  // XCD group x holds q + (x < r) blocks
  const int64_t x = bid & 7, k = bid >> 3;
  return x * q + (x < r ? x : r) + k;
}

// ======================================================= join: band order
// Band-major schedules.  A batch's queries draw their terms by df, so the big
// lists recur across it, and the queries' joins touch the same lists in the same
// url-id ranges: the bitmap words k_probe reads and the ranking records
// k_compact gathers.  In job order those re-reads are spread over the whole
// launch and all eight L2s.  k_order_hist and k_order_scatter counting-sort the
// step's tiles (ORDER_BUCKETS buckets), and k_probe / k_compact give every XCD
// group of blocks one contiguous slice of that order (xcd_slice), so the blocks
// resident on an XCD work on one url-id band and its L2 serves the re-reads:
//  * compaction: all tiles by the url id they start at (4096 bands): every list's
//    records of one band (C2: k_compact 268 -> 230 us, 11.7 -> 7.7 M lines read);
//  * probe: the probe tiles by 16 coarse url-id bands (every XCD sweeps its band
//    of every bitmap; 4 or 64 bands, or grouping by large list first, measured
//    slower: C3 k_probe 508 / 508 / 533 us per deferred step against 508, C2
//    123 / 123 / 114 against 115).
// Only the schedule changes: every tile writes its own slots.  Counting sort
// over G workgroups per order (LDS atomics run at about one lane per clock on a
// CU, so one workgroup took 30-35 us for C2's ~45k tiles): k_order_hist counts
// each workgroup's slice of tiles per bucket, k_order_scatter derives its
// slice's first slot per bucket from all the counts and places its tiles.
// Both orders run in the same two launches (OrderArgs: blocks of problem 0,
// then of problem 1).
constexpr int ORDER_BUCKETS = 4096;
constexpr int ORDER_THREADS = 1024;
__device__ __forceinline__ int order_bucket(uint32_t k, int shift) {
  return (int)min(k >> shift, (uint32_t)(ORDER_BUCKETS - 1));
}
__device__ __forceinline__ const OrderProb& order_prob(const OrderArgs& A, int& blk) {
  blk = (int)blockIdx.x;
  if (blk < A.p[0].nslices) return A.p[0];
  blk -= A.p[0].nslices;
  return A.p[1];
}
__global__ __launch_bounds__(ORDER_THREADS) void k_order_hist(OrderArgs A) {
  __shared__ int32_t cnt[ORDER_BUCKETS];
  int blk;
  const OrderProb& P = order_prob(A, blk);
  for (int i = threadIdx.x; i < ORDER_BUCKETS; i += ORDER_THREADS) cnt[i] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blk * P.slice, t1 = min(P.n, t0 + P.slice);
  for (int64_t t = t0 + threadIdx.x; t < t1; t += ORDER_THREADS) atomicAdd(&cnt[order_bucket(P.key[t], P.shift)], 1);
  __syncthreads();
  int4* h = reinterpret_cast<int4*>(P.hist + (int64_t)blk * ORDER_BUCKETS);
  h[threadIdx.x] = reinterpret_cast<const int4*>(cnt)[threadIdx.x];
}
__global__ __launch_bounds__(ORDER_THREADS) void k_order_scatter(OrderArgs A) {
  __shared__ int32_t cnt[ORDER_BUCKETS];
  __shared__ int32_t wsum[ORDER_THREADS / 64];
  static_assert(ORDER_BUCKETS == 4 * ORDER_THREADS, "four buckets per thread");
  int blk;
  const OrderProb& P = order_prob(A, blk);
  // buckets 4i..4i+3: totals over every slice, and the counts of the slices before this one
  int4 tot = make_int4(0, 0, 0, 0), pre = make_int4(0, 0, 0, 0);
  for (int w = 0; w < P.nslices; w++) {
    const int4 h = reinterpret_cast<const int4*>(P.hist + (int64_t)w * ORDER_BUCKETS)[threadIdx.x];
    tot.x += h.x; tot.y += h.y; tot.z += h.z; tot.w += h.w;
    if (w < blk) { pre.x += h.x; pre.y += h.y; pre.z += h.z; pre.w += h.w; }
  }
  const int32_t s = tot.x + tot.y + tot.z + tot.w;
  const int32_t inc = wave_incl_sum(s);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) wsum[wv] = inc;
  __syncthreads();
  int32_t off = inc - s;
  for (int w = 0; w < wv; w++) off += wsum[w];
  const int i4 = 4 * threadIdx.x;
  cnt[i4] = off + pre.x;
  cnt[i4 + 1] = off + tot.x + pre.y;
  cnt[i4 + 2] = off + tot.x + tot.y + pre.z;
  cnt[i4 + 3] = off + tot.x + tot.y + tot.z + pre.w;
  __syncthreads();
  const int64_t t0 = (int64_t)blk * P.slice, t1 = min(P.n, t0 + P.slice);
  for (int64_t t = t0 + threadIdx.x; t < t1; t += ORDER_THREADS) {
    const int32_t pos = atomicAdd(&cnt[order_bucket(P.key[t], P.shift)], 1);
    P.perm[pos] = make_int2((int32_t)t, P.tile_job[t]);
    if (P.pay_out) P.pay_out[pos] = P.pay[t];
  }
}

#ifndef YRWI_PROBE_LDS
#define YRWI_PROBE_LDS 4096
#endif
#define PROBE_LDS YRWI_PROBE_LDS  // large-list range (ids) a probe tile stages in LDS; 0: always gather

__device__ __forceinline__ int64_t lower_bound_uid(const uint32_t* __restrict__ u, int64_t lo, int64_t hi, uint32_t x) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ldg(u + mid) < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// lower bound of `key` in an index list with line heads: binary search over the
// level-2 heads (n/1024 ids, shared by every search of the list: L2 hits), then
// one line of level-1 heads and one leaf line
__device__ __forceinline__ int64_t lower_bound_list(const DList& L, uint32_t key) {
  const uint32_t* __restrict__ h2 = L.head + head1_cap(L.n);
  const int64_t n2 = head2_n(L.n);
  const int64_t a = lower_bound_uid(h2, 0, n2, key);  // first level-2 head >= key
  int64_t wl = a > 0 ? ((a - 1) << 10) + 1 : 0, wr = a < n2 ? (a << 10) : L.n;
  const int64_t f0 = (wl + 31) >> 5, f1 = (wr + 31) >> 5;
  const int64_t c = lower_bound_uid(L.head, f0, f1, key);
  if (c > f0) wl = ((c - 1) << 5) + 1;
  if (c < f1) wr = c << 5;
  return lower_bound_uid(L.uid, wl, wr, key);
}

#if PROBE_LDS > 0
// A probe tile whose large-list range [lo, hi) is longer than PROBE_LDS ids:
// the level-1 line heads of the range (first id of every 32-id line, DList::head)
// -- or, past PROBE_LDS of those, the level-2 heads (every 1024th id) -- are
// staged in LDS with one coalesced read, each key finds the first head >= it
// there, and the lower bound lies between that head and the one before: one
// line of level-1 heads (level 2 only) and one 128-B leaf line of ids per key,
// instead of a global binary search of log2(range) dependent loads.  Returns
// false (nothing read, no barrier) when the list has no heads or the range
// needs more than two levels; the decision is uniform over the workgroup.
// `kp` = the thread's small-list key (nullptr: no key).
__device__ __forceinline__ bool probe_heads(const DList& Lg, int64_t lo, int64_t hi, uint32_t* __restrict__ sL,
                                            uint32_t& key, const uint32_t* kp, int64_t* jl, bool* hit) {
  if (Lg.head == nullptr) return false;
  int sh = 5;
  const uint32_t* __restrict__ hd = Lg.head;
  int64_t g0 = (lo + 31) >> 5, g1 = (hi + 31) >> 5;  // heads at positions in [lo, hi)
  if (g1 - g0 > PROBE_LDS) {
    sh = 10;
    hd = Lg.head + head1_cap(Lg.n);
    g0 = (lo + 1023) >> 10;
    g1 = (hi + 1023) >> 10;
    if (g1 - g0 > PROBE_LDS) return false;
  }
  const int H = (int)(g1 - g0);
  for (int x = threadIdx.x; x < H; x += PROBE_TILE) sL[x] = hd[g0 + x];
  if (kp) key = *kp;
  __syncthreads();
  if (!kp) return true;
  int a = 0, b = H;  // first staged head >= key
  while (a < b) {
    const int mid = (a + b) >> 1;
    if (sL[mid] < key) a = mid + 1; else b = mid;
  }
  // the lower bound is in (position of head a-1, position of head a], within [lo, hi]
  int64_t wl = a > 0 ? ((g0 + a - 1) << sh) + 1 : lo;
  int64_t wr = a < H ? ((g0 + a) << sh) : hi;
  if (sh == 10) {  // narrow to one leaf line with the <= 32 level-1 heads inside [wl, wr)
    const int64_t f0 = (wl + 31) >> 5, f1 = (wr + 31) >> 5;
    const int64_t c = lower_bound_uid(Lg.head, f0, f1, key);
    if (c > f0) wl = ((c - 1) << 5) + 1;
    if (c < f1) wr = c << 5;
  }
  const int64_t p = lower_bound_uid(Lg.uid, wl, wr, key);
  *jl = p;
  *hit = p < hi && ldg(Lg.uid + p) == key;
  return true;
}
#endif

// A probe tile's BmFast: t >= 0 (k_probe_part) also decides whether the short
// path of k_probe serves the tile -- a bitmap probe of BM_TILE ids whose pairs
// are written with no exclusion mark, distance filter or chain test (the job's
// tiles, in whatever order k_probe takes them, read this and nothing else).
__device__ __forceinline__ BmFast bm_tile(const JoinQ& J, int64_t b, int64_t tile_base0, int64_t t) {
  BmFast F{};
  const DList& Sm = J.small_is_A ? J.A : J.B;
  const DList& Lg = J.small_is_A ? J.B : J.A;
  F.sm_uid = Sm.uid;
  F.lg_bm = Lg.bm;
  F.sm_n = Sm.n;
  F.s0 = (b - tile_base0) * (int64_t)J.ptile;
  F.src = J.pair_base + F.s0;
  F.t = t;
  F.flags = J.small_is_A ? BMF_SMALL_A : 0;
  if (t >= 0 && J.algo == JA_PROBE && Lg.bm && J.ptile == BM_TILE && J.mode != JM_MARK && J.maxd >= 65535 &&
      !J.chain_bm && !J.count_only)
    F.flags |= BMF_SIMPLE;
  return F;
}

__global__ void k_probe_part(const JoinQ* __restrict__ jobs, const int64_t* __restrict__ tile_base, int njobs,
                             int64_t tile0, int64_t ntiles, ProbeDesc* __restrict__ pdesc,
                             uint32_t* __restrict__ tile_key, int32_t* __restrict__ tile_job,
                             uint32_t* __restrict__ probe_key, int probe_shift, BmFast* __restrict__ fast) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const int j = find_job(tile_base, njobs, tile0 + t);
  const JoinQ& J = jobs[j];
  if (J.algo == JA_BMAND) {  // a range of bitmap units: no ids to read, no range
    const uint32_t id0 =
        (uint32_t)min((tile0 + t - tile_base[j]) * (int64_t)J.ptile * BM_UNIT_IDS, (int64_t)0xFFFFFFFF);
    if (tile_key) tile_key[tile0 + t] = id0;
    if (tile_job) tile_job[tile0 + t] = j;
    if (probe_key) probe_key[t] = id0 >> probe_shift;
    ProbeDesc D;
    D.job = j;
    D.pad = 0;
    D.lo = D.hi = 0;
    pdesc[t] = D;
    if (fast) fast[t] = bm_tile(J, tile0 + t, tile_base[j], t);
    return;
  }
  const DList& Sm = J.small_is_A ? J.A : J.B;
  const DList& Lg = J.small_is_A ? J.B : J.A;
  const int64_t s0 = (tile0 + t - tile_base[j]) * J.ptile;
  const int64_t s1 = s0 + J.ptile < Sm.n ? s0 + J.ptile : Sm.n;
  if (tile_key) tile_key[tile0 + t] = ldg(Sm.uid + s0);  // url id the tile starts at (k_order_hist / k_order_scatter)
  if (tile_job) tile_job[tile0 + t] = j;
  if (probe_key)  // (large list, 16 bands): k_probe's order
    probe_key[t] = ldg(Sm.uid + s0) >> probe_shift;  // 16 url-id bands: k_probe's order
  ProbeDesc D;
  D.job = j;
  D.pad = 0;
  if (fast) fast[t] = bm_tile(J, tile0 + t, tile_base[j], t);
  if (Lg.bm) {  // bitmap probe: no range needed
    D.lo = D.hi = 0;
    pdesc[t] = D;
    return;
  }
  const uint32_t k0 = ldg(Sm.uid + s0), k1 = ldg(Sm.uid + s1 - 1);
  if (Lg.head) {  // index list: through its line heads (level 2, one level-1 line, one leaf line)
    D.lo = lower_bound_list(Lg, k0);
    D.hi = lower_bound_list(Lg, k1 + 1u);  // ids < 2^32 - 1: k1 + 1 does not wrap
    pdesc[t] = D;
    return;
  }
  // lower bound of the first id, upper bound of the last
  int64_t lo0 = 0, hi0 = Lg.n, lo1 = 0, hi1 = Lg.n;
  while (lo0 < hi0 || lo1 < hi1) {
    if (lo0 < hi0) {
      const int64_t mid = (lo0 + hi0) >> 1;
      if (ldg(Lg.uid + mid) < k0) lo0 = mid + 1; else hi0 = mid;
    }
    if (lo1 < hi1) {
      const int64_t mid = (lo1 + hi1) >> 1;
      if (ldg(Lg.uid + mid) <= k1) lo1 = mid + 1; else hi1 = mid;
    }
  }
  D.lo = lo0;
  D.hi = lo1;
  pdesc[t] = D;
}

// Bitmap probe of one tile (k_probe): KPT small-list ids per thread, KPT * 256 per
// workgroup.  Deferred and exclusion steps with a small side of at least
// BM_LARGE_MIN ids take KPT = 8 (fewer, longer workgroups; their compaction
// gathers nothing: C3 k_probe 265 -> 243 us, k_compact 202 -> 180 with every
// long job at 8), the others KPT = 4 (a final step's compaction keeps its band
// order per tile: C2 at 8 took k_probe 111 -> 116 and k_compact 220 -> 237 us).
// T: the tile (its small list's ids, the large list's bitmap, its first small
// index and pair slot).  SIMPLE (a BmFast tile, built by k_probe_part: no
// exclusion mark, no distance filter, no chain test, pairs written) reads nothing
// of the job; otherwise J supplies those.
template <int KPT, bool SIMPLE>
__device__ __forceinline__ int32_t probe_bitmap(const BmFast& T, const JoinQ* Jp, int64_t b,
                                                uint2* __restrict__ pairs,
                                                uint32_t* __restrict__ pair_uid, int64_t* __restrict__ tile_src,
                                                int32_t* __restrict__ tile_cnt, int mark, uint64_t* sScan64,
                                                int32_t* tile_lvl = nullptr) {
  // url-id bitmap of the large list: one 16-B load per key (yrwi_bitmap.h) gives
  // membership and, for a hit, its list position (rank + bits below).  BM_TILE
  // small-list ids per tile, KPT per thread, lane-consecutive: key k*256 + tid, so
  // one load instruction's 64 lanes read 64 consecutive small-list ids and their
  // bitmap words fall into a few 128-B lines (thread-consecutive keys spread an
  // instruction over up to 64 lines: C2 k_probe 123 -> 114 us)
  static_assert(KPT <= 8, "bitmap tile: one 16-bit prefix field per key slot, four per 64-bit scan");
  const int64_t s0 = T.s0;
  const bool small_is_A = (T.flags & BMF_SMALL_A) != 0;
  const __amdgpu_buffer_rsrc_t rbm = bm_rsrc(T.lg_bm);
  uint32_t keys[KPT];
#pragma unroll
  for (int k = 0; k < KPT; k++) keys[k] = ldg(T.sm_uid + min(s0 + k * PROBE_TILE + (int64_t)threadIdx.x, T.sm_n - 1));
  // every bitmap load of the thread in flight at once: whole 16-B units through
  // buffer loads (a plain load was split, its second half loaded only on a hit,
  // and each key waited for the previous one)
  uint4 E[KPT];
#pragma unroll
  for (int k = 0; k < KPT; k++) E[k] = bm_unit(rbm, bm_at(keys[k]));
  uint32_t hm = 0;
  int32_t jls[KPT];  // large-list positions < 2^31
#pragma unroll
  for (int k = 0; k < KPT; k++) {
    jls[k] = 0;
    if (s0 + k * PROBE_TILE + (int64_t)threadIdx.x >= T.sm_n) continue;
    const BmAt a = bm_at(keys[k]);
    if (bm_test(a, E[k])) {
      hm |= 1u << k;
      jls[k] = bm_pos(a, E[k]);
    }
  }
  if (!SIMPLE) {
    const JoinQ& J = *Jp;
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      if (!((hm >> k) & 1u)) continue;
      const int64_t ik = s0 + k * PROBE_TILE + (int64_t)threadIdx.x;
      const int64_t ia = small_is_A ? ik : (int64_t)jls[k], ib = small_is_A ? (int64_t)jls[k] : ik;
      if (mark) {
        stg(J.removed + ia, (uint8_t)1);
      } else if (J.maxd < 65535 &&
                 joined_distance(J.A.feat + ia * FEAT_WORDS, J.B.feat + ib * FEAT_WORDS, J.mode) > J.maxd) {
        hm &= ~(1u << k);
      }
    }
    if (mark) return 0;
  }
  // a chained job's first later include list with a bitmap (JoinQ::chain_bm):
  // tested here on the hits, in registers, so that only its survivors are
  // written (with their rows in it) for k_chain; the tile's counts before and
  // after it are its first level counts
  const bool pre = !SIMPLE && Jp->chain_bm != nullptr && tile_lvl != nullptr;  // workgroup-uniform
  int32_t tp[KPT];
  uint32_t hm0 = hm;
  if (pre) {
    const __amdgpu_buffer_rsrc_t r2 = bm_rsrc(Jp->chain_bm);
    uint4 E2[KPT];
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      E2[k] = make_uint4(0, 0, 0, 0);
      if ((hm >> k) & 1u) E2[k] = bm_unit(r2, bm_at(keys[k]));
    }
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      const BmAt a = bm_at(keys[k]);
      tp[k] = bm_pos(a, E2[k]);  // list positions < 2^31
      if (!bm_test(a, E2[k])) hm &= ~(1u << k);
    }
  }
  // hits leave in key order (slot k's 256 keys, then slot k+1's): one 64-bit scan
  // of four 16-bit per-slot counts gives every hit's place in its slot
  constexpr int NSC = (KPT + 3) / 4;  // 64-bit scans of four slot counts each
  uint64_t ex[NSC], tot64[NSC];
#pragma unroll
  for (int q = 0; q < NSC; q++) {
    uint64_t cnt = 0;
#pragma unroll
    for (int k = 4 * q; k < KPT && k < 4 * q + 4; k++) cnt |= (uint64_t)((hm >> k) & 1u) << (16 * (k - 4 * q));
    ex[q] = block_excl_sum256_u64(cnt, sScan64, &tot64[q]);
  }
  const int64_t src = T.src;  // KPT * PROBE_TILE pair slots per tile
  int32_t base[KPT];
  int32_t run = 0;
#pragma unroll
  for (int k = 0; k < KPT; k++) {
    base[k] = run;
    run += (int32_t)((tot64[k / 4] >> (16 * (k % 4))) & 0xFFFFu);
  }
  if (threadIdx.x == 0) {
    tile_src[b] = src;
    tile_cnt[b] = run;
  }
  if (pre) {  // the tile's matches and those left after the prefix test
    uint64_t tot;
    block_excl_sum256_u64((uint64_t)__popc(hm0) | (uint64_t)__popc(hm) << 32, sScan64, &tot);
    if (threadIdx.x == 0) {
      int32_t* lv = tile_lvl + b * CHAIN_LVL;
      lv[0] = (int32_t)(tot & 0xFFFFFFFFu);
      lv[1] = (int32_t)(tot >> 32);
      for (int x = 0; x < Jp->chain_fill; x++) lv[2 + x] = lv[1];
    }
  }
  const bool write = SIMPLE || !Jp->count_only;  // workgroup-uniform
#pragma unroll
  for (int k = 0; k < KPT; k++) {
    if (!((hm >> k) & 1u)) continue;
    const int64_t ik = s0 + k * PROBE_TILE + (int64_t)threadIdx.x;
    const int64_t ia = small_is_A ? ik : (int64_t)jls[k], ib = small_is_A ? (int64_t)jls[k] : ik;
    const int32_t lo = base[k] + (int32_t)((ex[k / 4] >> (16 * (k % 4))) & 0xFFFFu);
    if (write) {
      pairs[src + lo] = make_uint2((uint32_t)ia, (uint32_t)ib);
      pair_uid[src + lo] = keys[k];
      if (pre) stg(Jp->chain_tup0 + src + lo, tp[k]);
    }
  }
  return run;
}




// MARK: an exclusion step (its own instantiation, so kernel traces tell the
// include steps' dispatches from the exclusion steps').  (Round 4 also built a
// CHAIN instantiation that kept a chained tile's matches in LDS and ran the chain
// tests in the same workgroup: C3 3.62 against 3.22-3.30 ms/step, DESIGN.md §3;
// removed in round 6.)
template <bool LONG, bool MARK>
__global__ __launch_bounds__(PROBE_TILE) void k_probe(const JoinQ* __restrict__ jobs,
                                                     const int64_t* __restrict__ tile_base,
                                                     const ProbeDesc* __restrict__ pdesc, int64_t tile0,
                                                     uint2* __restrict__ pairs, uint32_t* __restrict__ pair_uid,
                                                     int64_t* __restrict__ tile_src, int32_t* __restrict__ tile_cnt,
                                                     const int2* __restrict__ perm, int32_t* __restrict__ tile_lvl,
                                                     const BmFast* __restrict__ fast) {
  constexpr int mark = MARK ? 1 : 0;
  __shared__ int32_t sScan[4];
  __shared__ uint64_t sScan64[4];
#if PROBE_LDS > 0
  __shared__ uint32_t sL[PROBE_LDS];
#endif
  // the tile at this block's place in the schedule: its BmFast (same order as
  // perm) says whether the short path serves it -- one descriptor read before the
  // ids, instead of the order, the tile's descriptor and the job in turn
  const int64_t p = perm ? xcd_slice(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  int64_t t;
  if (!MARK && fast) {
    const BmFast F = fast[p];
    if (F.flags & BMF_SIMPLE) {
      probe_bitmap<BM_TILE / PROBE_TILE, true>(F, nullptr, tile0 + F.t, pairs, pair_uid, tile_src, tile_cnt, 0,
                                               sScan64);
      return;
    }
    t = F.t;
  } else {
    t = perm ? (int64_t)perm[p].x : p;
  }
  const int64_t b = tile0 + t;
  const ProbeDesc D = pdesc[t];
  const JoinQ& J = jobs[D.job];
  if (!MARK && J.algo == JA_BMAND) {  // workgroup-uniform: |A x B| from the bits of both bitmaps
    const int64_t w0 = (b - tile_base[D.job]) * (int64_t)J.ptile;
    const int64_t w1 = w0 + J.ptile < J.bm_words ? w0 + J.ptile : J.bm_words;
    const uint4* A = reinterpret_cast<const uint4*>(J.A.bm);
    const uint4* B = reinterpret_cast<const uint4*>(J.B.bm);
    int32_t c = 0;
    if (J.bm3) {
      const uint4* C = reinterpret_cast<const uint4*>(J.bm3);
      for (int64_t w = w0 + threadIdx.x; w < w1; w += PROBE_TILE) {
        const uint4 x = ldg(A + w), y = ldg(B + w), z = ldg(C + w);  // (w: the units' ranks)
        c += __popc(x.x & y.x & z.x) + __popc(x.y & y.y & z.y) + __popc(x.z & y.z & z.z);
      }
    } else {
      for (int64_t w = w0 + threadIdx.x; w < w1; w += PROBE_TILE) {
        const uint4 x = ldg(A + w), y = ldg(B + w);
        c += __popc(x.x & y.x) + __popc(x.y & y.y) + __popc(x.z & y.z);
      }
    }
    int32_t tot;
    block_excl_sum256(c, sScan, &tot);
    if (threadIdx.x == 0) {
      tile_src[b] = J.pair_base;
      tile_cnt[b] = tot;
    }
    return;
  }
  const DList& Sm = J.small_is_A ? J.A : J.B;
  const DList& Lg = J.small_is_A ? J.B : J.A;
  if (Lg.bm) {
    // a launch without long tiles does not carry the KPT_LARGE code (its registers
    // cost C2 a wave per SIMD: k_probe 111 -> 119 us)
    const BmFast T = bm_tile(J, b, tile_base[D.job], -1);
    if (LONG && J.ptile == KPT_LARGE * PROBE_TILE) {
      // (a job whose probe tests a chain list itself has BM_TILE tiles: layout_jobs)
      probe_bitmap<KPT_LARGE, false>(T, &J, b, pairs, pair_uid, tile_src, tile_cnt, mark, sScan64);
      return;
    }
    probe_bitmap<BM_TILE / PROBE_TILE, false>(T, &J, b, pairs, pair_uid, tile_src, tile_cnt, mark, sScan64, tile_lvl);
    return;
  }
  const int64_t s0 = (b - tile_base[D.job]) * PROBE_TILE;
  const int64_t i = s0 + threadIdx.x;
  bool hit = false;
  int64_t jl = 0;
  uint32_t key = 0;
#if PROBE_LDS > 0
  if (D.hi - D.lo <= PROBE_LDS) {  // workgroup-uniform
    const int64_t R = D.hi - D.lo;
    // short range: read it once, coalesced, and search in LDS -- 4 B per range
    // id instead of the two or three sector gathers per key of the lower levels
    const uint32_t* __restrict__ g = Lg.uid + D.lo;
    for (int x = threadIdx.x; x < (int)R; x += PROBE_TILE) sL[x] = g[x];
    if (i < Sm.n) key = ldg(Sm.uid + i);
    __syncthreads();
    if (i < Sm.n) {
      int lo = 0, hi = (int)R;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sL[mid] < key) lo = mid + 1; else hi = mid;
      }
      jl = D.lo + lo;
      hit = lo < (int)R && sL[lo] == key;
    }
  } else if (probe_heads(Lg, D.lo, D.hi, sL, key, i < Sm.n ? Sm.uid + i : nullptr, &jl, &hit)) {
    // long range of an index list: its line heads searched in LDS, one leaf line per key
  } else
#endif
  if (i < Sm.n) {
    // the upper levels of the 256 searches share lines of the range (L2 hits)
    key = ldg(Sm.uid + i);
    jl = lower_bound_uid(Lg.uid, D.lo, D.hi, key);
    hit = jl < D.hi && ldg(Lg.uid + jl) == key;
  }
  const int64_t ia = J.small_is_A ? i : jl, ib = J.small_is_A ? jl : i;
  if (hit && !mark && J.maxd < 65535) {
    if (joined_distance(J.A.feat + ia * FEAT_WORDS, J.B.feat + ib * FEAT_WORDS, J.mode) > J.maxd) hit = false;
  }
  if (mark) {
    if (hit) stg(J.removed + ia, (uint8_t)1);
    return;
  }
  // a chained job's first later include list with a bitmap: tested here (as in
  // probe_bitmap), only its survivors written, the tile's first two level counts
  const bool pre = J.chain_bm != nullptr && tile_lvl != nullptr;  // workgroup-uniform
  const bool hit0 = hit;
  int32_t tp = 0;
  if (pre && hit) {
    const __amdgpu_buffer_rsrc_t r2 = bm_rsrc(J.chain_bm);
    const BmAt a = bm_at(key);
    const uint4 E2 = bm_unit(r2, a);
    tp = bm_pos(a, E2);
    if (!bm_test(a, E2)) hit = false;
  }
  int32_t tot;
  const int32_t off = block_excl_sum256(hit ? 1 : 0, sScan, &tot);
  const int64_t src = J.pair_base + s0;  // PROBE_TILE pair slots per tile: the job's run is min(nA, nB) long
  if (threadIdx.x == 0) {
    tile_src[b] = src;
    tile_cnt[b] = tot;
  }
  if (pre) {
    int32_t tot0;
    block_excl_sum256(hit0 ? 1 : 0, sScan, &tot0);
    if (threadIdx.x == 0) {
      int32_t* lv = tile_lvl + b * CHAIN_LVL;
      lv[0] = tot0;
      lv[1] = tot;
      for (int x = 0; x < J.chain_fill; x++) lv[2 + x] = tot;
    }
    if (hit) stg(J.chain_tup0 + src + off, tp);
  }
  if (hit && !J.count_only) {
    pairs[src + off] = make_uint2((uint32_t)ia, (uint32_t)ib);
    pair_uid[src + off] = key;
  }
}

// ============================================================ join: scan
// tile_lvl (chained steps): a chained job's level counts (k_chain) summed into
// its ChainQ::level (pinned host memory, read after the step's synchronisation)
__global__ __launch_bounds__(256) void k_scan_tiles(const JoinQ* __restrict__ jobs,
                                                    const int64_t* __restrict__ tile_base,
                                                    const int32_t* __restrict__ tile_cnt,
                                                    int64_t* __restrict__ tile_off,
                                                    const int32_t* __restrict__ tile_lvl) {
  __shared__ int32_t sScan[4];
  __shared__ uint64_t sScan64[4];
  const JoinQ& J = jobs[blockIdx.x];
  const int64_t base = tile_base[blockIdx.x];
  const bool lvl = tile_lvl && J.chain;  // workgroup-uniform
  uint64_t acc[CHAIN_LVL] = {};
  int64_t running = 0;
  for (int64_t t0 = 0; t0 < J.ntiles; t0 += 256) {
    int64_t t = t0 + threadIdx.x;
    int32_t c = t < J.ntiles ? tile_cnt[base + t] : 0;
    if (lvl && t < J.ntiles)  // the level counts ride along (their loads in flight with the count's)
#pragma unroll
      for (int l = 0; l < CHAIN_LVL; l++) acc[l] += (uint64_t)tile_lvl[(base + t) * CHAIN_LVL + l];
    int32_t tot;
    int32_t ex = block_excl_sum256(c, sScan, &tot);
    if (t < J.ntiles) tile_off[base + t] = running + ex;
    running += tot;
  }
  if (threadIdx.x == 0 && J.m_out) *J.m_out = running;
  if (lvl) {
    int64_t* level = ldg(&J.chain->level);
    for (int l = 0; l < CHAIN_LVL; l++) {
      uint64_t tot;
      block_excl_sum256_u64(acc[l], sScan64, &tot);
      if (threadIdx.x == 0) level[l] = (int64_t)tot;
    }
  }
}

// Merge jobs: tile_src[t] = the job's pair_base + the exclusive prefix of its
// tiles' match bounds (k_partition), i.e. where each tile writes its pairs.
__global__ __launch_bounds__(256) void k_scan_bounds(const JoinQ* __restrict__ jobs,
                                                     const int64_t* __restrict__ tile_base,
                                                     int64_t* __restrict__ tile_src) {
  __shared__ int32_t sScan[4];
  const JoinQ& J = jobs[blockIdx.x];
  const int64_t base = tile_base[blockIdx.x];
  int64_t running = J.pair_base;
  for (int64_t t0 = 0; t0 < J.ntiles; t0 += 256) {
    const int64_t t = t0 + threadIdx.x;
    const int32_t c = t < J.ntiles ? (int32_t)tile_src[base + t] : 0;
    int32_t tot;
    const int32_t ex = block_excl_sum256(c, sScan, &tot);
    if (t < J.ntiles) tile_src[base + t] = running + ex;
    running += tot;
  }
}

// ============================================================ join: chain
// Chained folds (ChainQ, yrwi_internal.h): after a chained job's first step has
// written its matched pairs (tile slots), each pair is tested against the fold's
// later include lists and the exclusion lists; only the survivors stay in the
// tile's slots, with their rows in the later include lists.

// the ChainList of device memory through global loads (the struct reaches the
// kernel through a pointer held in device memory)
__device__ __forceinline__ ChainList load_cl(const ChainList* p) {
  ChainList L;
  L.uid = ldg(&p->uid);
  L.head = ldg(&p->head);
  L.bm = ldg(&p->bm);
  L.n = ldg(&p->n);
  return L;
}
__device__ __forceinline__ int64_t lower_bound_cl(const ChainList& L, uint32_t key) {
  if (!L.head) return lower_bound_uid(L.uid, 0, L.n, key);
  DList d{};
  d.uid = L.uid;
  d.head = L.head;
  d.n = L.n;
  return lower_bound_list(d, key);
}

// the range [lo, hi) of a list without a bitmap that holds the ids of a chain
// group's matches: one thread per (group, list), all groups in parallel (as
// k_probe_part), after the step's joins: the range spans the group's matches.
__global__ void k_chain_part(const JoinQ* __restrict__ jobs, const int64_t* __restrict__ tile_base, int njobs,
                             const int2* __restrict__ grp, int64_t n,
                             const uint32_t* __restrict__ pair_uid, const int64_t* __restrict__ tile_src,
                             const int32_t* __restrict__ tile_cnt, ProbeDesc* __restrict__ crange) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * CHAIN_MAXL) return;
  const int64_t u = i / CHAIN_MAXL;
  const int l = (int)(i % CHAIN_MAXL);
  const int2 G = grp[u];
  const int64_t t = G.x;
  const int j = find_job(tile_base, njobs, t);
  const JoinQ& J = jobs[j];
  const ChainQ* C = J.chain;
  if (!C || l >= ldg(&C->nl)) return;
  const ChainList L = load_cl(&C->l[l]);
  if (L.bm) return;
  int f = -1, e = -1;
  for (int k = 0; k < G.y; k++)
    if (tile_cnt[G.x + k] > 0) {
      if (f < 0) f = k;
      e = k;
    }
  if (f < 0) return;
  const uint32_t k0 = ldg(pair_uid + tile_src[G.x + f]);
  const uint32_t k1 = ldg(pair_uid + tile_src[G.x + e] + tile_cnt[G.x + e] - 1);
  ProbeDesc D;
  D.lo = lower_bound_cl(L, k0);
  D.hi = lower_bound_cl(L, k1 + 1u);  // ids < 2^32 - 1: no wrap
  D.job = j;
  D.pad = 0;
  crange[u * CHAIN_MAXL + l] = D;
}

#ifdef YRWI_CHAIN_PROF  // profiling build only: k_chain's paths (yrwi_chain_prof reads and clears them)
__device__ unsigned long long g_cprof[24];
#define CPROF(i, v) atomicAdd(&g_cprof[i], (unsigned long long)(v))
#else
#define CPROF(i, v)
#endif

// Lower bounds of up to KPT keys at once, each in its own window a[base, base + n)
// of at most 32 ids (a line of ids or of line heads): a power-of-two bisection of
// six rounds (results 0..32), the same for every key, with every live key's load
// of a round in flight together (the lines a per-key search would wait for one by one)
template <int KPT>
__device__ __forceinline__ void lower_bound_multi(const uint32_t* __restrict__ a, int64_t* base, int32_t* n,
                                                  const uint32_t* key, uint32_t live) {
  int32_t off[KPT];
#pragma unroll
  for (int k = 0; k < KPT; k++) off[k] = 0;
#pragma unroll
  for (int step = 32; step > 0; step >>= 1) {
    uint32_t v[KPT];
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      v[k] = 0xFFFFFFFFu;
      if (((live >> k) & 1u) && off[k] + step <= n[k]) v[k] = ldg(a + base[k] + off[k] + step - 1);
    }
#pragma unroll
    for (int k = 0; k < KPT; k++)
      if (v[k] < key[k]) off[k] += step;
  }
#pragma unroll
  for (int k = 0; k < KPT; k++) base[k] += off[k];
}

// the same in LDS over one array s[0, n) for every key (n <= 8192): the first
// index with s[i] >= key, no divergence (every key takes the same steps)
template <int KPT>
__device__ __forceinline__ void lds_lower_bound_multi(const uint32_t* s, int n, const uint32_t* key, uint32_t live,
                                                      int* out) {
#pragma unroll
  for (int k = 0; k < KPT; k++) out[k] = 0;
  int top = 1;
  while (top * 2 <= n) top *= 2;
  for (int step = n > 0 ? top : 0; step > 0; step >>= 1) {
#pragma unroll
    for (int k = 0; k < KPT; k++)
      if (((live >> k) & 1u) && out[k] + step <= n && s[out[k] + step - 1] < key[k]) out[k] += step;
  }
}

// Membership and position of the live keys (ascending, all inside [lo, hi)) in a
// list without a url-id bitmap, by the whole workgroup (barriers inside; every
// decision is workgroup-uniform): the range's ids staged in LDS when it fits;
// otherwise its level-1 line heads (every 32nd id) staged in LDS, an LDS search
// per key, then one leaf line of ids per key (lower_bound_multi); per-key head
// searches beyond that.
template <int KPT>
__device__ __forceinline__ void chain_search(const ChainList& L, int64_t lo, int64_t hi, const uint32_t* key,
                                             uint32_t live, int32_t* pos, uint32_t& hit, uint32_t* sL) {
  hit = 0;
  const int64_t R = hi - lo;
  __syncthreads();  // the previous list's stage is no longer read

  if (R <= PROBE_LDS) {
    CPROF(4, __popc(live));
    if (threadIdx.x == 0) CPROF(5, 1);
    for (int x = threadIdx.x; x < (int)R; x += 256) sL[x] = ldg(L.uid + lo + x);
    __syncthreads();
    int a[KPT];
    lds_lower_bound_multi<KPT>(sL, (int)R, key, live, a);
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      pos[k] = (int32_t)(lo + a[k]);
      if (((live >> k) & 1u) && a[k] < (int)R && sL[a[k]] == key[k]) hit |= 1u << k;
    }
    return;
  }
  if (L.head) {
    const int64_t g0 = (lo + 31) >> 5, g1 = (hi + 31) >> 5;  // level-1 heads at positions in [lo, hi)
    if (g1 - g0 <= PROBE_LDS) {  // workgroup-uniform
      CPROF(6, __popc(live));
      if (threadIdx.x == 0) CPROF(7, 1);
      const int H = (int)(g1 - g0);
      for (int x = threadIdx.x; x < H; x += 256) sL[x] = ldg(L.head + g0 + x);
      __syncthreads();
      int64_t wl[KPT];
      int32_t wn[KPT];
      int ha[KPT];  // first staged head >= key
      lds_lower_bound_multi<KPT>(sL, H, key, live, ha);
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        const int a = ha[k];
        // the lower bound lies in (position of head a-1, position of head a], within [lo, hi]
        wl[k] = a > 0 ? ((g0 + a - 1) << 5) + 1 : lo;
        const int64_t wr = a < H ? ((g0 + a) << 5) : hi;
        wn[k] = ((live >> k) & 1u) ? (int32_t)(wr - wl[k]) : 0;
      }
      lower_bound_multi<KPT>(L.uid, wl, wn, key, live);
      uint32_t v[KPT];
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        v[k] = 0xFFFFFFFFu;
        pos[k] = (int32_t)wl[k];
        if (((live >> k) & 1u) && wl[k] < hi) v[k] = ldg(L.uid + wl[k]);
      }
#pragma unroll
      for (int k = 0; k < KPT; k++)
        if (((live >> k) & 1u) && wl[k] < hi && v[k] == key[k]) hit |= 1u << k;
      return;
    }
  }
  // ranges past PROBE_LDS line heads (C3: 4 k of 100 M tests; a level-2 stage
  // here cost k_chain a wave per SIMD, 96 -> 106 VGPRs): per-key head searches
#pragma unroll
  for (int k = 0; k < KPT; k++) {
    pos[k] = 0;
    if (!((live >> k) & 1u)) continue;
    const int64_t q = lower_bound_cl(L, key[k]);
    pos[k] = (int32_t)q;
    if (q < L.n && ldg(L.uid + q) == key[k]) hit |= 1u << k;
  }
}

// The fold's later include lists and its exclusion lists, in order, against the
// live keys of a round (bitmap list: every live key's 16-B word in flight at once;
// otherwise chain_search over the range cr[l] staged / headed in LDS; barriers
// inside, every decision workgroup-uniform).  Returns the keys left alive; pos =
// their rows in the kept include lists; after1..3 = alive after include test 1..3.
template <int KPT>
__device__ __forceinline__ uint32_t chain_tests(const ChainList* cl, int ninc, int nl, int pos0,
                                                const ProbeDesc* cr, const uint32_t* key,
                                                uint32_t alive, int32_t (*pos)[KPT], uint32_t& after1,
                                                uint32_t& after2, uint32_t& after3, uint32_t* sL) {
  after1 = after2 = after3 = alive;
  for (int l = 0; l < nl; l++) {
    const ChainList L = cl[l];
    uint32_t hit = 0;
    int32_t p[KPT];
    if (L.bm) {
      CPROF(2, __popc(alive));
      if (threadIdx.x == 0) CPROF(3, 1);
      const __amdgpu_buffer_rsrc_t rbm = bm_rsrc(L.bm);
      uint4 E[KPT];
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        E[k] = make_uint4(0, 0, 0, 0);
        if ((alive >> k) & 1u) E[k] = bm_unit(rbm, bm_at(key[k]));
      }
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        const BmAt a = bm_at(key[k]);
        p[k] = bm_pos(a, E[k]);  // list positions < 2^31
        if (((alive >> k) & 1u) && bm_test(a, E[k])) hit |= 1u << k;
      }
    } else {
      const ProbeDesc D = cr[l];  // workgroup-uniform
      chain_search<KPT>(L, D.lo, D.hi, key, alive, p, hit, sL);
    }
    if (l < ninc) {
      alive &= hit;
      const int pi = l - pos0;  // the selection keeps no row
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        if (pi == 0) pos[0][k] = p[k];
        else if (pi == 1) pos[1][k] = p[k];
      }
      if (l == 0) after1 = alive;
      if (l == 1) after2 = alive;
      if (l == 2) after3 = alive;
    } else {
      alive &= ~hit;
    }
  }
  if (ninc < 2) after2 = after1;
  if (ninc < 3) after3 = after2;
  return alive;
}

constexpr int CHAIN_KPT = 3;  // matches per thread and round: 768 a round (one: 65 VGPRs, 7 waves, but C3 1.69 against 1.43 ms)
static_assert(CHAIN_KPT * 256 <= 1023, "k_chain: 10-bit count fields");

// One workgroup per chain group (up to CHAIN_GMAX consecutive tiles of one chained
// job, sized by the host to about one round of matches): the group's matches, in
// url-id order across its tiles (tile t's run, then tile t+1's), are tested in
// rounds of 768 (slot k*256 + tid of the round), list by list, only the live ones
// (the loads of a bitmap list all in flight at once); the survivors are written
// back to the front of their own tile's run, in order, with their rows in the
// later include lists.  A round reads only slots at or past every slot an earlier
// round wrote, and writes only slots it has read: in place.  The group's level
// counts (the fold's dispatch modes come from their sums per job) go to its first
// tile's tile_lvl, zeros to the others.  Few keys per thread keep the kernel at a
// high occupancy; whole groups of tiles per workgroup keep a probe step's sparse
// tiles (C3: ~90 matches per 2048-key tile) from costing a workgroup's dependent
// loads each.
__global__ __launch_bounds__(256) void k_chain(const JoinQ* __restrict__ jobs, const int64_t* __restrict__ tile_base,
                                               int njobs, const int2* __restrict__ grp,
                                               uint2* __restrict__ pairs, uint32_t* __restrict__ pair_uid,
                                               const int64_t* __restrict__ tile_src, int32_t* __restrict__ tile_cnt,
                                               int32_t* __restrict__ tile_lvl, const ProbeDesc* __restrict__ crange) {
  __shared__ uint32_t sL[PROBE_LDS];
  __shared__ uint64_t sScan64[4];
  __shared__ int32_t sOff[CHAIN_GMAX + 1];  // exclusive prefix of the tiles' match counts
  __shared__ int64_t sSrc[CHAIN_GMAX];
  __shared__ int32_t sRun[CHAIN_GMAX];      // survivors written so far, per tile
  __shared__ int32_t sCnt[CHAIN_GMAX];      // survivors of the round, per tile
  __shared__ int32_t sBase[CHAIN_GMAX];     // their exclusive prefix
  const int64_t g = blockIdx.x;
  const int2 G = grp[g];
  const int j = find_job(tile_base, njobs, G.x);
  const ChainQ* C = jobs[j].chain;
  const int tid = (int)threadIdx.x, n = G.y;
  __shared__ ChainList sCL[CHAIN_MAXL];  // the fold's lists and this group's ranges, loaded once
  __shared__ ProbeDesc sCR[CHAIN_MAXL];
  if (tid < 64) {
    const int32_t c = tid < n ? tile_cnt[G.x + tid] : 0;
    const int32_t inc = wave_incl_sum(c);
    if (tid < n) {
      sOff[tid + 1] = inc;
      sSrc[tid] = tile_src[G.x + tid];
      sRun[tid] = 0;
    }
    if (tid == 0) sOff[0] = 0;
  } else if (tid < 64 + CHAIN_MAXL) {
    sCL[tid - 64] = load_cl(&C->l[tid - 64]);
    sCR[tid - 64] = crange[g * CHAIN_MAXL + tid - 64];  // (unset for bitmap lists: unused)
  }
  __syncthreads();
  const int32_t M = sOff[n];
#ifdef YRWI_CHAIN_PROF
  const unsigned long long ck0 = wall_clock64();
  if (tid == 0) {
    CPROF(0, 1);
    CPROF(1, M);
    CPROF(12, n);
  }
#endif
  const int ninc = ldg(&C->ninc), nl = ldg(&C->nl), pos0 = ldg(&C->pos0), npos = ldg(&C->npos);
  const int pre = ldg(&C->pre);  // leading include tests the probe did (their rows in tup0, counts in tile_lvl)
  int32_t* tup0 = npos > 0 ? ldg(&C->tup[0]) : nullptr;
  int32_t* tup1 = npos > 1 ? ldg(&C->tup[1]) : nullptr;
  int32_t n1 = 0, n2 = 0, n3 = 0, nsurv = 0;  // live after include tests 1, 2, 3; survivors
  for (int r0 = 0; r0 < M; r0 += CHAIN_KPT * 256) {  // workgroup-uniform
    uint32_t key[CHAIN_KPT];
    uint2 pr[CHAIN_KPT];
    int32_t pos[CHAIN_MAXI][CHAIN_KPT];
    int32_t tk[CHAIN_KPT];  // the match's tile in the group
    uint32_t alive = 0;
#pragma unroll
    for (int k = 0; k < CHAIN_KPT; k++) {
      const int i = r0 + k * 256 + tid;
      key[k] = 0;
      pr[k] = make_uint2(0, 0);
      pos[0][k] = pos[1][k] = 0;
      tk[k] = 0;
      if (i < M) {
        int a = 0, b = n;  // last tile whose first match is at or before i
        while (b - a > 1) {
          const int m = (a + b) >> 1;
          if (sOff[m] <= i) a = m; else b = m;
        }
        tk[k] = a;
        const int64_t slot = sSrc[a] + (i - sOff[a]);
        key[k] = ldg(pair_uid + slot);
        pr[k] = ldg(reinterpret_cast<const uint2*>(pairs) + slot);
        if (pre) pos[0][k] = ldg(tup0 + slot);
        alive |= 1u << k;
      }
    }
    uint32_t after1, after2, after3;
    alive = chain_tests<CHAIN_KPT>(sCL + pre, ninc - pre, nl - pre, pos0 - pre, sCR + pre, key, alive, pos, after1,
                                   after2, after3, sL);
    if (tid < n) sCnt[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CHAIN_KPT; k++)
      if ((alive >> k) & 1u) atomicAdd(&sCnt[tk[k]], 1);
    // each survivor's rank in the round (slot order = the group's match order) and
    // the level counts, in 10-bit fields of one 64-bit scan (its barriers also
    // complete the LDS counts above)
    uint64_t c = (uint64_t)__popc(after1) << 30 | (uint64_t)__popc(after2) << 40 | (uint64_t)__popc(after3) << 50;
#pragma unroll
    for (int k = 0; k < CHAIN_KPT; k++) c |= (uint64_t)((alive >> k) & 1u) << (10 * k);
    uint64_t tot;
    const uint64_t ex = block_excl_sum256_u64(c, sScan64, &tot);
    if (tid == 0) {
      int32_t acc = 0;
      for (int x = 0; x < n; x++) {
        sBase[x] = acc;
        acc += sCnt[x];
      }
    }
    __syncthreads();
    int32_t before = 0;  // survivors of the round in earlier slots
#pragma unroll
    for (int k = 0; k < CHAIN_KPT; k++) {
      if ((alive >> k) & 1u) {
        const int x = tk[k];
        const int32_t rank = before + (int32_t)((ex >> (10 * k)) & 0x3FFu);
        const int64_t o = sSrc[x] + sRun[x] + (rank - sBase[x]);
        stg(reinterpret_cast<uint2*>(pairs) + o, pr[k]);
        stg(pair_uid + o, key[k]);
        if (tup0) stg(tup0 + o, pos[0][k]);
        if (tup1) stg(tup1 + o, pos[1][k]);
      }
      before += (int32_t)((tot >> (10 * k)) & 0x3FFu);
    }
    nsurv += before;
    n1 += (int32_t)((tot >> 30) & 0x3FFu);
    n2 += (int32_t)((tot >> 40) & 0x3FFu);
    n3 += (int32_t)((tot >> 50) & 0x3FFu);
    __syncthreads();  // every write of the round read sRun / sBase
    if (tid < n) sRun[tid] += sCnt[tid];
    __syncthreads();
  }
#ifdef YRWI_CHAIN_PROF
  if (tid == 0) {
    CPROF(13, (M + CHAIN_KPT * 256 - 1) / (CHAIN_KPT * 256));
    CPROF(15, wall_clock64() - ck0);
    CPROF(16, nsurv);
  }
#endif
  if (tid < n) {
    tile_cnt[G.x + tid] = sRun[tid];
    int32_t* lv = tile_lvl + (G.x + tid) * CHAIN_LVL;
    if (!pre) {
      lv[0] = tid == 0 ? M : 0;
      lv[1] = tid == 0 ? n1 : 0;
      lv[2] = tid == 0 ? n2 : 0;
      lv[3] = tid == 0 ? n3 : 0;
    } else if (ninc >= 2) {  // the probe wrote counts 0 and 1 per tile; this group's tests start at include 2
      lv[2] = tid == 0 ? n1 : 0;
      lv[3] = tid == 0 ? n2 : 0;
    }
    lv[4] = tid == 0 ? nsurv : 0;
  }
}


// ============================================================ url selection
// TermSearch's urlselection (yrwi_query_desc.urlselection): the selection's url
// ids from the dictionary, the size of every list of the query restricted to it,
// and (single include list) the restricted list itself.
__global__ void k_sel_lookup(const uint64_t* __restrict__ hi, const uint8_t* __restrict__ lo, int64_t n,
                             const uint64_t* __restrict__ dkhi, const uint8_t* __restrict__ dklo, int64_t nurls,
                             uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = hi[i];
  const uint8_t l = lo[i];
  int64_t a = 0, b = nurls;  // first dictionary key >= (h, l)
  while (a < b) {
    const int64_t mid = (a + b) >> 1;
    const uint64_t mh = ldg(dkhi + mid);
    if (mh < h || (mh == h && ldg(dklo + mid) < l)) a = mid + 1; else b = mid;
  }
  out[i] = (a < nurls && ldg(dkhi + a) == h && ldg(dklo + a) == l) ? (uint32_t)a : 0xFFFFFFFFu;
}

// membership (and position) of url id u in a list: its bitmap word, or its line heads
__device__ __forceinline__ bool list_has(const ChainList& L, uint32_t u, int64_t* pos) {
  if (L.n <= 0) return false;
  if (L.bm) {
    const BmAt a = bm_at(u);
    const uint4 U = ldg(reinterpret_cast<const uint4*>(L.bm) + a.unit);
    *pos = bm_pos(a, U);
    return bm_test(a, U);
  }
  const int64_t q = lower_bound_cl(L, u);
  *pos = q;
  return q < L.n && ldg(L.uid + q) == u;
}

__global__ __launch_bounds__(256) void k_sel_count(const SelCount* __restrict__ jobs) {
  __shared__ int32_t sScan[4];
  const SelCount& J = jobs[blockIdx.x];
  int32_t c = 0;
  for (int64_t i = threadIdx.x; i < J.nsel; i += 256) {
    int64_t p;
    c += list_has(J.L, ldg(J.sel + i), &p) ? 1 : 0;
  }
  int32_t tot;
  block_excl_sum256(c, sScan, &tot);
  if (threadIdx.x == 0) *J.out = tot;
}

__global__ __launch_bounds__(256) void k_sel_pick(const SelPick* __restrict__ jobs) {
  __shared__ int32_t sScan[4];
  const SelPick& J = jobs[blockIdx.x];
  int64_t run = 0;
  for (int64_t i0 = 0; i0 < J.nsel; i0 += 256) {  // the selection in url-id order: the list's order
    const int64_t i = i0 + threadIdx.x;
    int64_t p = 0;
    const bool h = i < J.nsel && list_has(J.L, ldg(J.sel + i), &p);
    int32_t tot;
    const int32_t off = block_excl_sum256(h ? 1 : 0, sScan, &tot);
    if (h) {
      const int64_t o = run + off;
      stg(J.out_uid + o, ldg(J.sel + i));
      store_rec(J.out_feat, o, load_rec(J.feat, p));
      // 40-B rows, 8-B aligned (index memory and arena allocations start on 256 B)
      const uint2* s2 = reinterpret_cast<const uint2*>(J.rows + p * YRWI_ROW_BYTES);
      uint2* d2 = reinterpret_cast<uint2*>(J.out_rows + o * YRWI_ROW_BYTES);
      for (int w = 0; w < YRWI_ROW_BYTES / 8; w++) stg(d2 + w, ldg(s2 + w));
    }
    run += tot;
  }
}

// ============================================================ join: compact
// Joined posting: J5 (WordReferenceVars.join :465-499) + J6 (toRowEntry :301-322
// -> WordReferenceRow ctor :116-161), on ranking records.  `o` is the record of
// the accumulated side (by-test modes: the large side's, joined with itself: its
// own features); b0/b1 are words 0-1 of the joined side (enumeration only).
__device__ __forceinline__ Rec joined_rec(Rec o, uint64_t b0, uint64_t b1, int mode, int64_t now_ms) {
  if (mode == JM_ENUM) {
    const uint64_t a0 = o.w[0], a1 = o.w[1];
    const int pa = (int)(a0 & 0xFFFF), pb = (int)(b0 & 0xFFFF);
    int pos = 0, post = pa;
    bool has = false;
    if (pa > 0 && pb > 0) {
      if (pa > pb) { pos = pa; post = pb; } else { pos = pb; }
      has = true;
    } else if (pa == 0) {
      post = pb;
    }
    const int oa = (int)((a1 >> 8) & 0xFF), ob = (int)((b1 >> 8) & 0xFF);
    int r = (int)(a1 & 0xFF), op = oa;
    if (oa == ob) r = min(r, (int)(b1 & 0xFF));
    else if (oa > ob) { op = ob; r = (int)(b1 & 0xFF); }
    const uint64_t w = max((a0 >> 16) & 0xFFFF, (b0 >> 16) & 0xFFFF);
    const uint64_t p = max((a0 >> 32) & 0xFFFF, (b0 >> 32) & 0xFFFF);
    const uint64_t u = max((a0 >> 48) & 0xFF, (b0 >> 48) & 0xFF);
    const uint64_t c = max(a0 >> 56, b0 >> 56);
    int dist = 0;
    if (has && post > 0) dist = post > pos ? post - pos : pos - post;
    if (dist == 0) dist = (int)((a1 >> 16) & 0xFF);
    o.w[0] = (uint64_t)post | w << 16 | p << 32 | u << 48 | c << 56;
    o.w[1] = (a1 & ~0xFFFFFFull) | (uint64_t)r | (uint64_t)op << 8 | (uint64_t)(dist & 0xFF) << 16;  // i: 1-byte cell
  }
  // lastModified re-encoded through MicroDate: future days clamp to today (J6)
  const int32_t mddlm = clamp_days((int32_t)(o.w[2] & 0xFFFF), now_ms);
  o.w[2] = (o.w[2] & ~0xFFFFull) | (uint64_t)(mddlm & 0xFFFF);
  return o;
}

// One workgroup per COMPACT_TILES consecutive tiles: the tiles' matches are
// concatenated (LDS prefix of their counts) and spread over all 256 threads.
// The output url id comes with the pair (written by k_join / k_probe).  Each
// thread takes COMPACT_UNROLL matches at a time and issues all their pair and
// record loads before combining any of them: the gathers are latency-bound, so
// more of them in flight per thread is what moves the records.  Per match it
// gathers the 32-byte record of the accumulated side (one aligned 32-B block)
// and words 0-1 of the joined side (16 B), and writes one 32-B record + url id.
#ifndef YRWI_COMPACT_TILES
#define YRWI_COMPACT_TILES 4
#endif
// 2 since the chained folds' fold_chain (round 4): compaction 0.307 -> 0.227 ms
// on C3, 3.02 -> 2.95 on C4, 0.226 -> 0.213 on C2 against 4; 8 matches per
// thread 0.629 / 4.41 / 0.238 (profiles/archive/r04_compact_sweep.txt).
#ifndef YRWI_COMPACT_UNROLL
#define YRWI_COMPACT_UNROLL 2
#endif
constexpr int COMPACT_TILES = YRWI_COMPACT_TILES;
constexpr int COMPACT_UNROLL = YRWI_COMPACT_UNROLL;

struct CompactJob {
  const uint64_t* af;
  const uint64_t* bf;
  uint64_t* ofeat;
  uint32_t* ouid;
  int64_t now_ms;
  int64_t off;
  int64_t src;  // the tile's run in the pair arrays
  int32_t mode;
  int32_t atw;           // A deferred: its rows' source width (0: A has records)
  const int32_t* atup;
  int32_t* otup;         // deferred output (otw > 0)
  const FoldSrc* fold;   // A deferred, this the last step: the fold's lists and modes
  int32_t otw;
  int32_t bw;            // words per posting of bf (FEAT_WORDS, or 2 for an enumeration's DList::j5)
  int32_t ctw;           // chained job: lists of the fold (0: not chained)
  int32_t cperm;         // count-first fold: pair = (row in list 2, row in list 0), ctup0 / ctup1 = rows in lists 1 / 3
  const int32_t* ctup0;  // chained job: rows in the fold's lists 2 and 3 (ChainQ::tup)
  const int32_t* ctup1;
};

// the record of a deferred row (sources r[0..tw-1] in the fold's lists): J5/J6
// folded step by step, as every step's k_compact would have materialised it
__device__ __forceinline__ Rec fold_deferred(const FoldSrc& F, const int32_t* __restrict__ r, int tw, int64_t now_ms) {
  Rec acc = load_rec(F.feat[0], r[0]);
  for (int s = 0; s + 1 < tw; s++) {
    const int32_t m = F.mode[s];
    const int64_t e = r[s + 1];
    ulonglong2 b = make_ulonglong2(0, 0);
    if (m == JM_TEST_LARGE_B) acc = load_rec(F.feat[s + 1], e);  // self-join of the larger side
    else if (m == JM_ENUM)
      b = F.j5[s + 1] ? ldg(reinterpret_cast<const ulonglong2*>(F.j5[s + 1]) + e)
                      : ldg(reinterpret_cast<const ulonglong2*>(F.feat[s + 1] + e * FEAT_WORDS));
    acc = joined_rec(acc, b.x, b.y, m, now_ms);
  }
  return acc;
}

// the record of a chained fold's survivor (rows r0..r3 in the fold's lists 0..tw-1):
// J5/J6 step by step over all tw lists, with each step's dispatch mode
__device__ __forceinline__ Rec fold_chain(const FoldSrc* F, int32_t r0, int32_t r1, int32_t r2, int32_t r3, int tw,
                                          int64_t now_ms) {
  Rec acc = load_rec(ldg(&F->feat[0]), r0);
#pragma unroll
  for (int s = 0; s < 2 + CHAIN_MAXI - 1; s++) {
    if (s + 1 >= tw) break;
    const int32_t m = ldg(&F->mode[s]);
    const int64_t e = s == 0 ? r1 : s == 1 ? r2 : r3;
    ulonglong2 b = make_ulonglong2(0, 0);
    if (m == JM_TEST_LARGE_B) {
      acc = load_rec(ldg(&F->feat[s + 1]), e);  // self-join of the larger side
    } else if (m == JM_ENUM) {
      const uint64_t* j5 = ldg(&F->j5[s + 1]);
      b = j5 ? ldg(reinterpret_cast<const ulonglong2*>(j5) + e)
             : ldg(reinterpret_cast<const ulonglong2*>(ldg(&F->feat[s + 1]) + e * FEAT_WORDS));
    }
    acc = joined_rec(acc, b.x, b.y, m, now_ms);
  }
  return acc;
}

// CHAIN: the step has chained jobs (k_chain ran): their matches fold the records
// of all the fold's lists (fold_chain) instead of joining A's record with B's
template <bool CHAIN>
__global__ __launch_bounds__(256) void k_compact(const JoinQ* __restrict__ jobs, const int64_t* __restrict__ tile_base,
                                                 int njobs, int64_t ntiles, const uint2* __restrict__ pairs,
                                                 const uint32_t* __restrict__ pair_uid,
                                                 const int64_t* __restrict__ tile_src,
                                                 const int32_t* __restrict__ tile_cnt,
                                                 const int64_t* __restrict__ tile_off,
                                                 const int2* __restrict__ perm,
                                                 const int32_t* __restrict__ tile_job, int skip_sum) {
  __shared__ int32_t sPre[COMPACT_TILES + 1];
  __shared__ CompactJob sJ[COMPACT_TILES];
  // band order (k_order_hist / k_order_scatter): this block's tiles are positions p0.. of the sorted order
  const int64_t p0 = (perm ? xcd_slice(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x) * COMPACT_TILES;
  if (threadIdx.x < 64) {
    const int64_t p = p0 + threadIdx.x;
    int32_t c = 0;
    if (threadIdx.x < COMPACT_TILES && p < ntiles) {
      // tile and job: one load in band order (k_order_scatter packs them)
      int64_t t = p;
      int j;
      if (perm) {
        const int2 tj = perm[p];
        t = tj.x;
        j = tj.y;
      } else {
        j = tile_job ? tile_job[t] : find_job(tile_base, njobs, t);
      }
      c = tile_cnt[t];
      if (c && jobs[j].count_only) c = 0;  // a count-first fold's counted join: nothing to compact
      if (c && skip_sum && jobs[j].psum) c = 0;  // compacted by k_compact_sum
      if (c) {
        const JoinQ& J = jobs[j];
        CompactJob& X = sJ[threadIdx.x];
        X.af = J.A.feat;
        X.bf = J.mode == JM_ENUM && J.B.j5 ? J.B.j5 : J.B.feat;
        X.bw = J.mode == JM_ENUM && J.B.j5 ? 2 : FEAT_WORDS;
        X.ofeat = J.out_feat;
        X.ouid = J.out_uid;
        X.now_ms = J.now_ms;
        X.off = tile_off[t];
        X.src = tile_src[t];
        X.mode = J.mode;
        X.atw = J.A.tup ? J.A.tw : 0;
        X.atup = J.A.tup;
        X.otup = J.out_tup;
        X.otw = J.out_tup ? J.out_tw : 0;
        X.fold = J.fold;
        X.ctw = 0;
        X.cperm = 0;
        if (CHAIN && J.chain) {
          const int ni = ldg(&J.chain->npos);
          X.ctw = 2 + ni;
          X.cperm = ldg(&J.chain->perm);
          X.ctup0 = ni > 0 ? ldg(&J.chain->tup[0]) : nullptr;
          X.ctup1 = ni > 1 ? ldg(&J.chain->tup[1]) : nullptr;
        }
      }
    }
    const int32_t inc = wave_incl_sum(c);
    if (threadIdx.x < COMPACT_TILES) sPre[threadIdx.x + 1] = inc;
    if (threadIdx.x == 0) sPre[0] = 0;
  }
  __syncthreads();
  const int32_t total = sPre[COMPACT_TILES];
  for (int m0 = threadIdx.x; m0 < total; m0 += COMPACT_UNROLL * 256) {
    int tl[COMPACT_UNROLL];
    int64_t pi[COMPACT_UNROLL];
    uint2 pr[COMPACT_UNROLL];
    uint32_t uid[COMPACT_UNROLL];
#pragma unroll
    for (int u = 0; u < COMPACT_UNROLL; u++) {
      const int m = m0 + u * 256;
      tl[u] = -1;
      if (m < total) {
        int lo = 0, hi = COMPACT_TILES - 1;  // largest lt with sPre[lt] <= m
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (sPre[mid] <= m) lo = mid; else hi = mid - 1;
        }
        tl[u] = lo;
        pi[u] = sJ[lo].src + (m - sPre[lo]);
        pr[u] = pairs[pi[u]];
        uid[u] = pair_uid[pi[u]];
      }
    }
    // deferred rows: a step before the fold's last writes the joined row's sources
    // (A's sources + the B row) instead of gathering any record
#pragma unroll
    for (int u = 0; u < COMPACT_UNROLL; u++) {
      if (tl[u] < 0) continue;
      const CompactJob& X = sJ[tl[u]];
      if (X.otw == 0) continue;
      const int64_t o = X.off + (m0 + u * 256 - sPre[tl[u]]);
      int32_t* dst = X.otup + o * X.otw;
      if (X.atw) {
        const int32_t* srcr = X.atup + (int64_t)pr[u].x * X.atw;
        for (int j = 0; j < X.atw; j++) stg(dst + j, ldg(srcr + j));
      } else {
        stg(dst, (int32_t)pr[u].x);
      }
      stg(dst + X.otw - 1, (int32_t)pr[u].y);
      stg(X.ouid + o, uid[u]);
      tl[u] = -1;
    }
    Rec A[COMPACT_UNROLL];
    ulonglong2 B[COMPACT_UNROLL];
    // one record (the accumulated side's; a by-test step's larger side's; a
    // deferred side's fold) and the joined side's 12 J5 bytes per match, the
    // gathers of all COMPACT_UNROLL matches in flight together (a 16-B load of the
    // joined side left its top dword dead, the compiler reused that register and
    // the next gather waited; a second, branch-free loop for steps without
    // deferred sides cost 4-10 %: more registers for both)
#pragma unroll
    for (int u = 0; u < COMPACT_UNROLL; u++) {
      B[u] = make_ulonglong2(0, 0);
      if (tl[u] < 0) continue;
      const CompactJob& X = sJ[tl[u]];
      if (CHAIN && X.ctw) {
        const int32_t t2 = X.ctw > 2 ? ldg(X.ctup0 + pi[u]) : 0;
        A[u] = X.cperm == 2 ? fold_chain(X.fold, (int32_t)pr[u].y, t2, ldg(X.ctup1 + pi[u]), (int32_t)pr[u].x,
                                         X.ctw, X.now_ms)
               : X.cperm ? fold_chain(X.fold, (int32_t)pr[u].y, t2, (int32_t)pr[u].x,
                                      X.ctw > 3 ? ldg(X.ctup1 + pi[u]) : 0, X.ctw, X.now_ms)
                       : fold_chain(X.fold, (int32_t)pr[u].x, (int32_t)pr[u].y, t2,
                                    X.ctw > 3 ? ldg(X.ctup1 + pi[u]) : 0, X.ctw, X.now_ms);
        continue;
      }
      if (X.mode == JM_TEST_LARGE_B) A[u] = load_rec(X.bf, pr[u].y);
      else if (X.atw) A[u] = fold_deferred(*X.fold, X.atup + (int64_t)pr[u].x * X.atw, X.atw, X.now_ms);
      else A[u] = load_rec(X.af, pr[u].x);
      if (X.mode == JM_ENUM) B[u] = ldg_j5(X.bf + (int64_t)pr[u].y * X.bw);
    }
#pragma unroll
    for (int u = 0; u < COMPACT_UNROLL; u++) {
      if (tl[u] < 0) continue;
      const CompactJob& X = sJ[tl[u]];
      const int64_t o = X.off + (m0 + u * 256 - sPre[tl[u]]);
      store_rec(X.ofeat, o, (CHAIN && X.ctw) ? A[u] : joined_rec(A[u], B[u].x, B[u].y, X.mode, X.now_ms));
      stg(X.ouid + o, uid[u]);
    }
  }
}

// url-hash key -> the 12 url-hash characters (Base64Order.enhancedCoder alphabet)
__device__ __forceinline__ uint8_t b64char(uint32_t c) {
  return (uint8_t)(c < 26 ? 'A' + c : c < 52 ? 'a' + (c - 26) : c < 62 ? '0' + (c - 52) : c == 62 ? '-' : '_');
}
__device__ __forceinline__ void key_chars(uint64_t hi, uint32_t lo, uint8_t* h) {
#pragma unroll
  for (int j = 0; j < 10; j++) h[j] = b64char((uint32_t)(hi >> (4 + 6 * (9 - j))) & 63u);
  h[10] = b64char((uint32_t)(((hi & 15u) << 2) | ((lo >> 6) & 3u)));
  h[11] = b64char(lo & 63u);
}

// url-hash key of a row (bytes 0..11), as k_validate computes it for the index
__device__ __forceinline__ void row_key(const Row& r, uint64_t& hi, uint32_t& lo) {
  uint64_t x = 0;
#pragma unroll
  for (int j = 0; j < 10; j++) x = (x << 6) | (uint64_t)(ahpla(r.b(j)) & 63);
  const uint32_t c10 = (uint32_t)ahpla(r.b(10)) & 63, c11 = (uint32_t)ahpla(r.b(11)) & 63;
  hi = (x << 4) | (c10 >> 2);
  lo = ((c10 & 3u) << 6) | c11;
}

// ranking records of index rows (built with the url dictionary)
__global__ void k_features(const uint8_t* __restrict__ rows, int64_t n, uint64_t* __restrict__ feat) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) store_rec(feat, i, rec_of_row(load_row(rows + i * YRWI_ROW_BYTES)));
}

// joined container -> the 40-byte rows toRowEntry writes (WordReferenceRow ctor
// :116-161): url hash from the dictionary, freshUntil = lastModified + 2 (today -
// lastModified) days, floored at 0; typeofword and reserve 0
__global__ void k_feat_rows(const uint64_t* __restrict__ feat, const uint32_t* __restrict__ uid,
                            const uint64_t* __restrict__ dkhi, const uint8_t* __restrict__ dklo, int64_t n,
                            int64_t now_ms, uint8_t* __restrict__ rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Rec q = load_rec(feat, i);
  uint8_t h[12];
  key_chars(dkhi[uid[i]], dklo[uid[i]], h);
  Row r{};
  for (int j = 0; j < 12; j++) r.set(j, h[j]);
  const uint64_t w0 = q.w[0], w1 = q.w[1], w2 = q.w[2];
  const int32_t a = (int32_t)(w2 & 0xFFFF);
  int32_t fresh = add32(a, mul32(sub32(micro_date_days(now_ms), a), 2));
  if (fresh < 0) fresh = 0;
  r.set(O_A, (uint32_t)a >> 8); r.set(O_A + 1, (uint32_t)a);
  r.set(O_S, (uint32_t)fresh >> 8); r.set(O_S + 1, (uint32_t)fresh);
  r.set(O_U, (uint32_t)(w0 >> 48));
  r.set(O_W, (uint32_t)(w0 >> 24)); r.set(O_W + 1, (uint32_t)(w0 >> 16));
  r.set(O_P, (uint32_t)(w0 >> 40)); r.set(O_P + 1, (uint32_t)(w0 >> 32));
  r.set(O_D, (uint32_t)(w1 >> 56));
  r.set(O_L, (uint32_t)(w2 >> 16)); r.set(O_L + 1, (uint32_t)(w2 >> 24));
  r.set(O_X, (uint32_t)(w1 >> 24)); r.set(O_Y, (uint32_t)(w1 >> 32));
  r.set(O_M, (uint32_t)(w1 >> 40)); r.set(O_N, (uint32_t)(w1 >> 48));
  r.set(O_G, 0);
  for (int j = 0; j < 4; j++) r.set(O_Z + j, (uint32_t)(w2 >> (32 + 8 * j)));
  r.set(O_C, (uint32_t)(w0 >> 56));
  r.set(O_T, (uint32_t)(w0 >> 8)); r.set(O_T + 1, (uint32_t)w0);
  r.set(O_R, (uint32_t)w1); r.set(O_O, (uint32_t)(w1 >> 8)); r.set(O_I, (uint32_t)(w1 >> 16));
  r.set(O_K, 0);
  store_row(rows + i * YRWI_ROW_BYTES, r);
}

// ================================================================ ranking

__device__ __forceinline__ uint64_t host36(const Row& r) {
  uint64_t h = 0;
#pragma unroll
  for (int j = 6; j < 12; j++) h = (h << 6) | (uint64_t)(ahpla(r.b(j)) & 63);
  return h;
}
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int32_t wave_max_i(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int32_t wave_min_i(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int32_t wave_sum_i(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_min_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}

constexpr int32_t BIG = 0x7FFFFFFF;

// Two 16-bit fields per word: min / max of both halves at once (v_pk_min_u16 /
// v_pk_max_u16); every int field of a record fits 16 bits.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_max16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
constexpr int NP2 = (NF + 1) / 2;  // packed field pairs

// termFrequency c / d (WordReferenceRow.java:355-357) as an exact fraction: c <= 255,
// 1 <= d < 2^17, so c1 * d2 < 2^25 compares two of them without rounding, and the
// double of the extreme fraction is the extreme double (division rounds monotonically)
__device__ __forceinline__ bool frac_lt(int32_t c1, int32_t d1, int32_t c2, int32_t d2) { return c1 * d2 < c2 * d1; }


// 2048 slots (16 KB of LDS for keys and counts) for a bucket of ~512 postings:
// k_hbucket on C5 custom 32.3 us with 4096, 28.5 with 2048, 30.2 with 1024 (the
// fuller table probes longer); buckets above the target spill to the global table
#ifndef YRWI_HB_LOG2
#define YRWI_HB_LOG2 11
#endif
constexpr int HB_LOG2 = YRWI_HB_LOG2;
constexpr int HB_SLOTS = 1 << HB_LOG2;  // LDS table slots of a bucket
__device__ __forceinline__ uint32_t hp_bucket(uint32_t hid, int32_t nb) {
  uint32_t x = hid * 0x9E3779B1u;
  x ^= x >> 15;
  x *= 0x85EBCA77u;
  x ^= x >> 13;
  return (uint32_t)(((uint64_t)x * (uint64_t)nb) >> 32);
}


// One workgroup per CHUNK container elements.  Rows are read coalesced
// (element s*256 + tid of the chunk), which is all the order-independent parts
// need (min/max, tf, host counts); the order-dependent fold of posintext /
// distance works on thread-consecutive elements, so (valid, p, od) of every
// element are exchanged through LDS.
//
// Authority host counts (ReferenceOrder doms / maxdomcount, :176-216): every
// valid element adds one to its host's slot in the query's global table.  (Round
// 4 tried the host hash in the record's word 3 instead of ByteArray.hashCode:
// C5 custom k_reduce 121.7 -> 97.9 us, but the candidates' hashCode then came
// from the url keys, C2 k_score 94 -> 115 us -- the headline pays for it; and a
// separate per-chunk kernel counting in LDS first, k_hostcount: 107 + 18 us, its
// distinct (chunk, host) pairs still cost a device atomic each.)
__global__ __launch_bounds__(CHUNK_THREADS) void k_reduce(const RankQ* __restrict__ qs,
                                                         const int32_t* __restrict__ chunk_q,
                                                         ChunkSum* __restrict__ out, ShardSum* __restrict__ shard) {
  __shared__ int32_t sI[4 * (2 * NF + 8)];
  __shared__ int32_t sScan[4];
  __shared__ int32_t sFirst[4];
  // element order: valid << 31 | od << 16 | p; one pad word per 32 so that the
  // thread-consecutive reads (stride CHUNK_IPT words) spread over the banks
  __shared__ uint32_t sPO[CHUNK + CHUNK / 32];
  __shared__ uint32_t sSegP[SEGC];  // the first SEGC fold segments (more: the summary overflows)
  __shared__ uint32_t sSegM[SEGC];
  __shared__ uint32_t sSegL[SEGC];
  __shared__ int32_t sFirstInfo[3];
  extern __shared__ int32_t sHB[];  // authority by partition: the chunk's elements per host bucket (dynamic)

  const int64_t b = blockIdx.x;
  const int qi = chunk_q[b];
  const RankQ& Q = qs[qi];
  if (Q.pieces) return;  // the compaction summarised this query (k_compact_sum)
  const int64_t c = b - Q.chunk_base;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int hnb = Q.ecnt ? Q.hp_nb : 0;  // block-uniform
  for (int i = threadIdx.x; i < hnb; i += CHUNK_THREADS) sHB[i] = 0;
  if (hnb) __syncthreads();

  // ---- coalesced pass: order-independent summaries
  uint32_t pmn[NP2], pmx[NP2];  // fields 2j | 2j+1 << 16
#pragma unroll
  for (int j = 0; j < NP2; j++) { pmn[j] = 0xFFFFFFFFu; pmx[j] = 0u; }
  int32_t pmax = -1, nval = 0, myfirst = BIG;
  int32_t hmax = 0;  // largest host count this thread saw (one atomicMax per wave below)
  int32_t tcn = -1, tdn = 1, tcx = -1, tdx = 1;  // tf min / max as fractions (-1: none yet)
  int32_t av[CHUNK_IPT];  // lastModified days of my elements (-1: invalid)
  // RED_GROUP elements at a time: their exclusion marks, then their records, all
  // in flight together (in bounds whatever the element: the last row stands in
  // past the end), so a thread waits for memory twice per group, not per element
  constexpr int RED_GROUP = 4;
  bool vg[RED_GROUP];
  Rec rg[RED_GROUP];
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++) {
    const int eo = s * CHUNK_THREADS + (int)threadIdx.x;
    const int64_t e = c * CHUNK + eo;
    if (s % RED_GROUP == 0) {
#pragma unroll
      for (int u = 0; u < RED_GROUP; u++) vg[u] = e + (int64_t)u * CHUNK_THREADS < Q.n;
      uint8_t mk[RED_GROUP];
#pragma unroll
      for (int u = 0; u < RED_GROUP; u++) {
        const int64_t eu = min(e + (int64_t)u * CHUNK_THREADS, Q.n - 1);
        mk[u] = Q.removed ? ldg(Q.removed + eu) : (uint8_t)0;
        rg[u] = load_rec(Q.feat, eu);
      }
#pragma unroll
      for (int u = 0; u < RED_GROUP; u++) vg[u] = vg[u] & (mk[u] == 0);
    }
    const bool v = vg[s % RED_GROUP];
    av[s] = -1;
    uint32_t po = 0;
    if (v) {
      const Feat F = decode_rec(rg[s % RED_GROUP]);
#pragma unroll
      for (int j = 0; j < NP2; j++) {
        const uint32_t w = (uint32_t)F.f[2 * j] | (2 * j + 1 < NF ? (uint32_t)F.f[2 * j + 1] << 16 : 0u);
        pmn[j] = pk_min16(pmn[j], w);
        pmx[j] = pk_max16(pmx[j], w);
      }
      {
        const int32_t tc = F.f[F_HITCOUNT], td = F.f[F_WORDSINTEXT] + F.f[F_WORDSINTITLE] + 1;
        if (tcn < 0 || frac_lt(tc, td, tcn, tdn)) { tcn = tc; tdn = td; }
        if (tcx < 0 || frac_lt(tcx, tdx, tc, td)) { tcx = tc; tdx = td; }
      }
      pmax = max(pmax, F.p);
      nval++;
      myfirst = min(myfirst, eo);
      av[s] = F.a;
      po = 0x80000000u | ((uint32_t)F.od << 16) | (uint32_t)F.p;
      if (hnb) atomicAdd(&sHB[hp_bucket((uint32_t)(rg[s % RED_GROUP].w[3] >> 34), hnb)], 1);
      if (Q.want_authority && !Q.ecnt) {  // (a partitioned query: k_hbucket counts)
        const uint64_t key = elem_host(Q, rg[s % RED_GROUP].w[3], e) + 1;
        uint64_t slot = mix64(key) & Q.hmask;
        while (true) {
          // (a plain read before the compare-and-swap, to skip it for hosts already
          // in: k_reduce 99 -> 158 us on C5 custom, the read's round trip first)
          const unsigned long long prev =
              atomicCAS((unsigned long long*)&Q.hkeys[slot], 0ull, (unsigned long long)key);
          if (prev == 0ull || prev == key) {
            const uint32_t cnt = atomicAdd(&Q.hcnt[slot], 1u) + 1u;
            hmax = max(hmax, (int32_t)cnt);  // the last increment of every host sees its final count
            break;
          }
          slot = (slot + 1) & Q.hmask;
        }
      }
    }
    sPO[eo + (eo >> 5)] = po;
  }
  if (Q.want_authority && !Q.ecnt) {  // block-uniform: one atomicMax per wave instead of one per posting
    const int32_t wm = wave_max_i(hmax);
    if (lane == 0 && wm > 0) atomicMax(&shard[qi].maxdom, wm);
  }
  if (hnb) {  // the chunk's bucket counts (bucket-major), for k_hpart_scatter's scan
    __syncthreads();
    for (int i = threadIdx.x; i < hnb; i += CHUNK_THREADS) Q.hp_hist[Q.hp_hoff + (int64_t)i * Q.nchunks + c] = sHB[i];
  }
  // first valid element of the chunk (element order)
  int32_t firstIdx;
  {
    int32_t v = wave_min_i(myfirst);
    if (lane == 0) sFirst[wv] = v;
    __syncthreads();  // also publishes sPO
    v = min(min(sFirst[0], sFirst[1]), min(sFirst[2], sFirst[3]));
    __syncthreads();
    firstIdx = v;
  }
  // virtualAge over the rest (the chunk's first element is min/max's clone candidate)
  int32_t vamn = BIG, vamx = -1;
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++) {
    const int eo = s * CHUNK_THREADS + (int)threadIdx.x;
    if (av[s] >= 0 && eo != firstIdx) { vamn = min(vamn, av[s]); vamx = max(vamx, av[s]); }
    if (eo == firstIdx) sFirstInfo[2] = av[s];
  }

  // ---- ordered pass on thread-consecutive elements: local fold segments
  // (records of the prefix max of posintext over the rest)
  bool rest[CHUNK_IPT];
  int32_t P[CHUNK_IPT], OD[CHUNK_IPT];
  int32_t pmax_rest = -1;
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++) {
    const int eo = (int)threadIdx.x * CHUNK_IPT + s;
    const uint32_t po = sPO[eo + (eo >> 5)];
    P[s] = (int32_t)(po & 0xFFFFu);
    OD[s] = (int32_t)((po >> 16) & 0xFFu);
    rest[s] = (po >> 31) && eo != firstIdx;
    if (rest[s]) pmax_rest = max(pmax_rest, P[s]);
    if (eo == firstIdx) { sFirstInfo[0] = P[s]; sFirstInfo[1] = OD[s]; }
  }
  const int32_t lpin = block_excl_max256(pmax_rest, sScan);
  bool isrec[CHUNK_IPT];
  int32_t LP = lpin, nrec = 0;
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++) {
    isrec[s] = rest[s] && P[s] > LP;
    if (isrec[s]) { LP = P[s]; nrec++; }
  }
  // backward pass: per record, max od and the last positive od (keyed by element
  // position so that a max over keys selects the latest one)
  int32_t recM[CHUNK_IPT];
  uint32_t recL[CHUNK_IPT];
  int32_t accM = 0;
  uint32_t accL = 0;
#pragma unroll
  for (int s = CHUNK_IPT - 1; s >= 0; s--) {
    recM[s] = 0;
    recL[s] = 0;
    if (rest[s]) {
      accM = max(accM, OD[s]);
      if (accL == 0 && OD[s] > 0)
        accL = (((uint32_t)threadIdx.x * CHUNK_IPT + (uint32_t)s + 1u) << 8) | (uint32_t)OD[s];
    }
    if (isrec[s]) {
      recM[s] = accM;
      recL[s] = accL;
      accM = 0;
      accL = 0;
    }
  }
  int32_t nsegTot;
  int32_t segOff = block_excl_sum256(nrec, sScan, &nsegTot);
  // the first SEGC segments in LDS (a chunk with more keeps none: its summary
  // overflows and k_shard_fin rewalks it)
  int32_t segM = 0, segL = 0;  // this thread's share of M_rest / L_rest (max over every segment)
  {
    int32_t o = segOff;
#pragma unroll
    for (int s = 0; s < CHUNK_IPT; s++) {
      if (isrec[s]) {
        if (o < SEGC) {
          sSegP[o] = (uint32_t)P[s];
          sSegM[o] = (uint32_t)recM[s];
          sSegL[o] = recL[s];
        }
        segM = max(segM, recM[s]);
        segL = max(segL, (int32_t)recL[s]);
        o++;
      }
    }
  }
  __syncthreads();
  // the continuation piece (elements before this thread's first record) belongs to segment segOff-1
  if (segOff > 0 && (accM > 0 || accL > 0)) {
    if (segOff - 1 < SEGC) {
      atomicMax(&sSegM[segOff - 1], (uint32_t)accM);
      if (accL > 0) atomicMax(&sSegL[segOff - 1], accL);
    }
    segM = max(segM, accM);
    segL = max(segL, (int32_t)accL);
  }
  __syncthreads();

  // block reductions: packed min/max pairs, the int summaries, the tf fractions
  constexpr int NI = 2 * NP2 + 6 + 4;
  int32_t vals[NI];
#pragma unroll
  for (int j = 0; j < NP2; j++) {
    uint32_t x = pmn[j], y = pmx[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      x = pk_min16(x, (uint32_t)__shfl_xor((int)x, o, 64));
      y = pk_max16(y, (uint32_t)__shfl_xor((int)y, o, 64));
    }
    vals[j] = (int32_t)x;
    vals[NP2 + j] = (int32_t)y;
  }
  vals[2 * NP2 + 0] = wave_min_i(vamn);
  vals[2 * NP2 + 1] = wave_max_i(vamx);
  vals[2 * NP2 + 2] = wave_max_i(pmax);
  vals[2 * NP2 + 3] = wave_sum_i(nval);
  vals[2 * NP2 + 4] = wave_max_i(segM);
  vals[2 * NP2 + 5] = wave_max_i(segL);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t c1 = __shfl_xor(tcn, o, 64), d1 = __shfl_xor(tdn, o, 64);
    const int32_t c2 = __shfl_xor(tcx, o, 64), d2 = __shfl_xor(tdx, o, 64);
    if (c1 >= 0 && (tcn < 0 || frac_lt(c1, d1, tcn, tdn))) { tcn = c1; tdn = d1; }
    if (c2 >= 0 && (tcx < 0 || frac_lt(tcx, tdx, c2, d2))) { tcx = c2; tdx = d2; }
  }
  vals[2 * NP2 + 6] = tcn;
  vals[2 * NP2 + 7] = tdn;
  vals[2 * NP2 + 8] = tcx;
  vals[2 * NP2 + 9] = tdx;
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NI; i++) sI[wv * NI + i] = vals[i];
  }
  __syncthreads();
  // the four waves combined in parallel, one summary field per thread.  A query
  // of one chunk gets its shard summary here too (the chunk's summary is the
  // shard's; its fold pieces are the chunk's segments) unless the segments
  // overflowed -- k_shard_fin skips it then (one = true).
  ChunkSum& S = out[b];
  const int t = (int)threadIdx.x;
  int32_t nvb = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) nvb += sI[w * NI + 2 * NP2 + 3];
  const bool one = Q.nchunks == 1 && nsegTot <= SEGC;
  ShardSum& SS = shard[qi];
  if (t < NP2) {  // field pair t: min
    uint32_t x = 0xFFFFFFFFu;
    for (int w = 0; w < 4; w++) x = pk_min16(x, (uint32_t)sI[w * NI + t]);
    S.mn[2 * t] = nvb ? (int32_t)(x & 0xFFFFu) : BIG;
    if (2 * t + 1 < NF) S.mn[2 * t + 1] = nvb ? (int32_t)(x >> 16) : BIG;
    if (one) {
      SS.mn[2 * t] = S.mn[2 * t];
      if (2 * t + 1 < NF) SS.mn[2 * t + 1] = S.mn[2 * t + 1];
    }
  } else if (t < 2 * NP2) {  // field pair t - NP2: max
    const int j = t - NP2;
    uint32_t y = 0u;
    for (int w = 0; w < 4; w++) y = pk_max16(y, (uint32_t)sI[w * NI + NP2 + j]);
    S.mx[2 * j] = nvb ? (int32_t)(y & 0xFFFFu) : -1;
    if (2 * j + 1 < NF) S.mx[2 * j + 1] = nvb ? (int32_t)(y >> 16) : -1;
    if (one) {
      SS.mx[2 * j] = S.mx[2 * j];
      if (2 * j + 1 < NF) SS.mx[2 * j + 1] = S.mx[2 * j + 1];
    }
  } else if (t == 2 * NP2) {
    int32_t a = BIG, z = -1, pm = -1, Mr = 0, Lk = 0;
    for (int w = 0; w < 4; w++) {
      a = min(a, sI[w * NI + 2 * NP2]);
      z = max(z, sI[w * NI + 2 * NP2 + 1]);
      pm = max(pm, sI[w * NI + 2 * NP2 + 2]);
      Mr = max(Mr, sI[w * NI + 2 * NP2 + 4]);
      Lk = max(Lk, sI[w * NI + 2 * NP2 + 5]);
    }
    S.va_mn_rest = a;
    S.va_mx_rest = z;
    S.pmax = pm;
    S.nvalid = nvb;
    S.M_rest = Mr;
    S.L_rest = (int32_t)((uint32_t)Lk & 0xFFu);
    S.nseg = nsegTot;
    S.overflow = nsegTot > SEGC ? 1 : 0;
    if (one) {
      SS.nvalid = nvb;
      SS.va_mn_rest = a;
      SS.va_mx_rest = z;
      SS.nseg = nvb ? nsegTot : 0;
      SS.overflow = 0;
    }
  } else if (t == 2 * NP2 + 1) {
    int32_t cn = -1, dn = 1, cx = -1, dx = 1;
    for (int w = 0; w < 4; w++) {
      const int32_t c1 = sI[w * NI + 2 * NP2 + 6], d1 = sI[w * NI + 2 * NP2 + 7];
      const int32_t c2 = sI[w * NI + 2 * NP2 + 8], d2 = sI[w * NI + 2 * NP2 + 9];
      if (c1 >= 0 && (cn < 0 || frac_lt(c1, d1, cn, dn))) { cn = c1; dn = d1; }
      if (c2 >= 0 && (cx < 0 || frac_lt(cx, dx, c2, d2))) { cx = c2; dx = d2; }
    }
    // the same double WordReferenceRow.termFrequency computes (decode_rec)
    S.tf_mn = cn >= 0 ? (double)cn / (double)dn : 1e300;
    S.tf_mx = cx >= 0 ? (double)cx / (double)dx : -1e300;
    if (one) {
      SS.tf_mn = S.tf_mn;
      SS.tf_mx = S.tf_mx;
    }
  } else if (t == 2 * NP2 + 2) {
    S.end = (int32_t)min((int64_t)(c + 1) * CHUNK, Q.n);
    if (firstIdx != BIG) {
      S.first = (int32_t)(c * CHUNK + firstIdx);
      S.p_first = sFirstInfo[0];
      S.od_first = sFirstInfo[1];
      S.a_first = sFirstInfo[2];
    } else {
      S.first = -1;
      S.p_first = S.od_first = S.a_first = 0;
    }
    if (one) {
      SS.has_first = nvb > 0;
      SS.p_first = S.p_first;
      SS.od_first = S.od_first;
      SS.a_first = S.a_first;
    }
  } else if (t >= 64 && t < 64 + SEGC) {
    const int i = t - 64;
    if (nsegTot <= SEGC && i < nsegTot) {
      S.seg[i] = (sSegP[i] << 16) | ((sSegM[i] & 0xFFu) << 8) | (sSegL[i] & 0xFFu);
      if (one && nvb) SS.seg[i] = S.seg[i];
    }
  }
}

// ---------------------------------------------- compaction with summary pieces
// The last step of queries whose containers need no pass but the normalisation
// (JoinQ::psum: no exclusion marks, no authority counts): one wave per tile, the
// tile's matches in order, 64 x COMPACT_UNROLL at a time, the same records and
// url ids as k_compact, and the tile's ChunkSum -- what k_reduce
// computes for a chunk (ReferenceOrder NormalizeWorker :163-210, see k_reduce),
// here over the tile's run of the container [tile_off, tile_off + cnt), every
// element of it valid -- from the records it has in registers, so the rank phase
// does not read the container back for it (k_piece_merge / k_shard_fin fold the
// pieces in tile order).  The step's other jobs go through k_compact (skip_sum),
// among them the chained folds with exclusions inside the chain: their survivors
// are sparse in their tiles (C3 1.23 -> 1.37 ms/step through this kernel), and
// k_compact packs four tiles per workgroup.  CHAIN: the step has chained jobs.
template <bool CHAIN>
__global__ __launch_bounds__(64) void k_compact_sum(const JoinQ* __restrict__ jobs,
                                                    const int64_t* __restrict__ tile_base, int njobs, int64_t ntiles,
                                                    const uint2* __restrict__ pairs,
                                                    const uint32_t* __restrict__ pair_uid,
                                                    const int64_t* __restrict__ tile_src,
                                                    const int32_t* __restrict__ tile_cnt,
                                                    const int64_t* __restrict__ tile_off, const int2* __restrict__ perm,
                                                    const int32_t* __restrict__ tile_job) {
  const int lane = threadIdx.x;
  // band order (k_order_hist / k_order_scatter): this wave's tile is position p of the sorted order
  const int64_t p = perm ? xcd_slice(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  if (p >= ntiles) return;
  int64_t t = p;
  int j;
  if (perm) {
    const int2 tj = perm[p];
    t = tj.x;
    j = tj.y;
  } else {
    j = tile_job ? tile_job[t] : find_job(tile_base, njobs, t);
  }
  const JoinQ& J = jobs[j];
  if (!J.psum) return;  // (k_compact's)
  const int32_t cnt = tile_cnt[t];
  const int64_t off = tile_off[t];
  ChunkSum* __restrict__ S = J.psum + (t - tile_base[j]);
  if (cnt == 0) {
    if (lane == 0) {
      S->nvalid = 0;
      S->first = -1;
      S->end = (int32_t)off;
      S->nseg = 0;
      S->overflow = 0;
    }
    return;
  }
  const uint64_t* afeat = J.A.feat;
  const uint64_t* bfeat = J.mode == JM_ENUM && J.B.j5 ? J.B.j5 : J.B.feat;
  const int32_t bw = J.mode == JM_ENUM && J.B.j5 ? 2 : FEAT_WORDS;
  const int32_t mode = J.mode;
  const int32_t atw = J.A.tup ? J.A.tw : 0;
  const int32_t* atup = J.A.tup;
  const FoldSrc* fold = J.fold;
  uint64_t* ofeat = J.out_feat;
  uint32_t* ouid = J.out_uid;
  const int64_t now_ms = J.now_ms;
  const int64_t src = tile_src[t];
  // a chained fold's survivors (k_chain): the records of all the fold's lists (fold_chain)
  int32_t ctw = 0, cperm = 0;
  const int32_t *ctup0 = nullptr, *ctup1 = nullptr;
  if (CHAIN && J.chain) {
    const int ni = ldg(&J.chain->npos);
    ctw = 2 + ni;
    cperm = ldg(&J.chain->perm);
    ctup0 = ni > 0 ? ldg(&J.chain->tup[0]) : nullptr;
    ctup1 = ni > 1 ? ldg(&J.chain->tup[1]) : nullptr;
  }
  // summary state: order-independent parts per lane, the ordered fold wave-uniform
  uint32_t pmn[NP2], pmx[NP2];  // fields 2j | 2j+1 << 16
#pragma unroll
  for (int k = 0; k < NP2; k++) { pmn[k] = 0xFFFFFFFFu; pmx[k] = 0u; }
  int32_t pmax = -1, tcn = -1, tdn = 1, tcx = -1, tdx = 1, vamn = BIG, vamx = -1;
  int32_t mrest = 0, lkey = 0;  // over the rest: max stored distance, (position + 1) << 8 | last positive one
  int32_t pf = 0, of = 0, af = 0;  // the tile's first element (lane 0)
  int32_t prun = -1, nseg = 0, segP = 0, segM = 0, segK = 0;  // prefix max of the rest; the open segment
  // Software pipeline, one group = 64 x COMPACT_UNROLL matches: while group g's
  // summary runs, group g+1's gathers are in flight and group g+2's pairs loaded
  // (the summary's arithmetic would otherwise sit between the wave's gathers).
  uint2 npr[COMPACT_UNROLL];
  uint32_t nuid[COMPACT_UNROLL], uid[COMPACT_UNROLL];
  Rec A[COMPACT_UNROLL];
  ulonglong2 B[COMPACT_UNROLL];
  auto load_pairs = [&](int32_t g0) {
#pragma unroll
    for (int u = 0; u < COMPACT_UNROLL; u++) {
      const int32_t m = g0 + u * 64 + lane;
      if (m < cnt) {
        npr[u] = pairs[src + m];
        nuid[u] = pair_uid[src + m];
      }
    }
  };
  auto gather = [&](int32_t g0) {  // from npr (group g0's pairs); uid takes nuid
#pragma unroll
    for (int u = 0; u < COMPACT_UNROLL; u++) {
      B[u] = make_ulonglong2(0, 0);
      uid[u] = nuid[u];
      if (g0 + u * 64 + lane >= cnt) continue;
      const uint2 pr = npr[u];
      if (CHAIN && ctw) {
        const int64_t pi = src + g0 + u * 64 + lane;
        const int32_t t2 = ctw > 2 ? ldg(ctup0 + pi) : 0;
        A[u] = cperm == 2 ? fold_chain(fold, (int32_t)pr.y, t2, ldg(ctup1 + pi), (int32_t)pr.x, ctw, now_ms)
               : cperm    ? fold_chain(fold, (int32_t)pr.y, t2, (int32_t)pr.x, ctw > 3 ? ldg(ctup1 + pi) : 0,
                                       ctw, now_ms)
                          : fold_chain(fold, (int32_t)pr.x, (int32_t)pr.y, t2, ctw > 3 ? ldg(ctup1 + pi) : 0,
                                       ctw, now_ms);
        continue;
      }
      if (mode == JM_TEST_LARGE_B) A[u] = load_rec(bfeat, pr.y);
      else if (atw) A[u] = fold_deferred(*fold, atup + (int64_t)pr.x * atw, atw, now_ms);
      else A[u] = load_rec(afeat, pr.x);
      if (mode == JM_ENUM) B[u] = ldg_j5(bfeat + (int64_t)pr.y * bw);
    }
  };
  load_pairs(0);
  gather(0);
  load_pairs(COMPACT_UNROLL * 64);
  for (int32_t m0 = 0; m0 < cnt; m0 += COMPACT_UNROLL * 64) {
    Rec Rg[COMPACT_UNROLL];
#pragma unroll
    for (int u = 0; u < COMPACT_UNROLL; u++) {
      const int32_t m = m0 + u * 64 + lane;
      if (m < cnt) {
        Rg[u] = (CHAIN && ctw) ? A[u] : joined_rec(A[u], B[u].x, B[u].y, mode, now_ms);
        store_rec(ofeat, off + m, Rg[u]);
        stg(ouid + off + m, uid[u]);
      }
    }
    if (m0 + COMPACT_UNROLL * 64 < cnt) {  // (wave-uniform) the next group's gathers, the one after's pairs
      gather(m0 + COMPACT_UNROLL * 64);
      load_pairs(m0 + 2 * COMPACT_UNROLL * 64);
    }
#pragma unroll
    for (int u = 0; u < COMPACT_UNROLL; u++) {
      const int32_t m = m0 + u * 64 + lane;  // the element's place in the tile
      const bool okm = m < cnt;
      const Rec& R = Rg[u];
      // ---- the summary over these 64 elements, in order
      int32_t P = -1, OD = 0;
      const bool rest = okm && m > 0;
      if (okm) {
        const Feat F = decode_rec(R);
#pragma unroll
        for (int k = 0; k < NP2; k++) {
          const uint32_t w = (uint32_t)F.f[2 * k] | (2 * k + 1 < NF ? (uint32_t)F.f[2 * k + 1] << 16 : 0u);
          pmn[k] = pk_min16(pmn[k], w);
          pmx[k] = pk_max16(pmx[k], w);
        }
        const int32_t tc = F.f[F_HITCOUNT], td = F.f[F_WORDSINTEXT] + F.f[F_WORDSINTITLE] + 1;
        if (tcn < 0 || frac_lt(tc, td, tcn, tdn)) { tcn = tc; tdn = td; }
        if (tcx < 0 || frac_lt(tcx, tdx, tc, td)) { tcx = tc; tdx = td; }
        pmax = max(pmax, F.p);
        P = F.p;
        OD = F.od;
        if (m == 0) {
          pf = F.p;
          of = F.od;
          af = F.a;
        } else {
          vamn = min(vamn, F.a);
          vamx = max(vamx, F.a);
          mrest = max(mrest, F.od);
          if (F.od > 0) lkey = max(lkey, ((m + 1) << 8) | F.od);
        }
      }
      // records: rest elements above the prefix max of the rest before them
      const int32_t incl = wave_incl_max(rest ? P : -1);
      const int32_t pex = max(lane == 0 ? -1 : __shfl_up(incl, 1, 64), prun);
      const bool isrec = rest && P > pex;
      const uint64_t heads = __ballot(isrec);
      // per segment: max stored distance, (position + 1) << 8 | the last positive one
      // (a segmented inclusive scan headed at the records)
      int32_t sm = rest ? OD : 0;
      int32_t sk = (rest && OD > 0) ? ((m + 1) << 8) | OD : 0;
      bool hd = isrec;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t m2 = __shfl_up(sm, o, 64), k2 = __shfl_up(sk, o, 64);
        const bool h2 = __shfl_up((int)hd, o, 64) != 0;
        if (lane >= o && !hd) { sm = max(sm, m2); sk = max(sk, k2); hd = h2; }
      }
      // the lanes before the first record continue the open segment
      const int pre_end = heads ? __ffsll((long long)heads) - 2 : 63;
      if (pre_end >= 0 && nseg > 0) {
        segM = max(segM, __shfl(sm, pre_end, 64));
        segK = max(segK, __shfl(sk, pre_end, 64));
      }
      uint64_t hm = heads;
      while (hm) {  // wave-uniform
        const int r = __ffsll((long long)hm) - 1;
        hm &= hm - 1;
        const int end = hm ? __ffsll((long long)hm) - 2 : 63;
        if (nseg > 0 && nseg <= SEGC && lane == 0)
          S->seg[nseg - 1] = ((uint32_t)segP << 16) | (((uint32_t)segM & 0xFFu) << 8) | ((uint32_t)segK & 0xFFu);
        nseg++;
        segP = __shfl(P, r, 64);
        segM = __shfl(sm, end, 64);
        segK = __shfl(sk, end, 64);
      }
      prun = max(prun, __shfl(incl, 63, 64));
    }
  }
  if (nseg > 0 && nseg <= SEGC && lane == 0)
    S->seg[nseg - 1] = ((uint32_t)segP << 16) | (((uint32_t)segM & 0xFFu) << 8) | ((uint32_t)segK & 0xFFu);
  // the wave's reductions; lane i writes field i
#pragma unroll
  for (int k = 0; k < NP2; k++) {
    uint32_t x = pmn[k], y = pmx[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      x = pk_min16(x, (uint32_t)__shfl_xor((int)x, o, 64));
      y = pk_max16(y, (uint32_t)__shfl_xor((int)y, o, 64));
    }
    pmn[k] = x;
    pmx[k] = y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t c1 = __shfl_xor(tcn, o, 64), d1 = __shfl_xor(tdn, o, 64);
    const int32_t c2 = __shfl_xor(tcx, o, 64), d2 = __shfl_xor(tdx, o, 64);
    if (c1 >= 0 && (tcn < 0 || frac_lt(c1, d1, tcn, tdn))) { tcn = c1; tdn = d1; }
    if (c2 >= 0 && (tcx < 0 || frac_lt(tcx, tdx, c2, d2))) { tcx = c2; tdx = d2; }
  }
  pmax = wave_max_i(pmax);
  vamn = wave_min_i(vamn);
  vamx = wave_max_i(vamx);
  mrest = wave_max_i(mrest);
  lkey = wave_max_i(lkey);
  pf = __shfl(pf, 0, 64);
  of = __shfl(of, 0, 64);
  af = __shfl(af, 0, 64);
#pragma unroll
  for (int k = 0; k < NP2; k++) {
    if (lane == k) {
      S->mn[2 * k] = (int32_t)(pmn[k] & 0xFFFFu);
      S->mx[2 * k] = (int32_t)(pmx[k] & 0xFFFFu);
      if (2 * k + 1 < NF) {
        S->mn[2 * k + 1] = (int32_t)(pmn[k] >> 16);
        S->mx[2 * k + 1] = (int32_t)(pmx[k] >> 16);
      }
    }
  }
  if (lane == 16) {
    S->nvalid = cnt;
    S->first = (int32_t)off;
    S->end = (int32_t)(off + cnt);
    S->p_first = pf;
    S->od_first = of;
    S->a_first = af;
    S->pmax = pmax;
  } else if (lane == 17) {
    S->M_rest = mrest;
    S->L_rest = (int32_t)((uint32_t)lkey & 0xFFu);
    S->va_mn_rest = vamn;
    S->va_mx_rest = vamx;
    S->nseg = nseg;
    S->overflow = nseg > SEGC ? 1 : 0;
  } else if (lane == 18) {
    // the same double WordReferenceRow.termFrequency computes (decode_rec)
    S->tf_mn = (double)tcn / (double)tdn;
    S->tf_mx = (double)tcx / (double)tdx;
  }
}

// ------------------------------------------------- fold piece bookkeeping
struct SegList {
  uint32_t* seg;
  int32_t cap;
  int32_t n;
  int32_t overflow;
  int32_t prun;  // running prefix max of the rest (-1: none yet)
  __device__ void add(int32_t P, int32_t M, int32_t L) {
    if (P > prun) {
      if (n < cap) seg[n] = ((uint32_t)P << 16) | ((uint32_t)M << 8) | (uint32_t)L;
      else overflow = 1;
      n++;
      prun = P;
    } else if (n > 0 && n <= cap) {
      uint32_t s = seg[n - 1];
      uint32_t m = max((s >> 8) & 0xFFu, (uint32_t)M);
      uint32_t l = L > 0 ? (uint32_t)L : (s & 0xFFu);
      seg[n - 1] = (s & 0xFFFF0000u) | (m << 8) | l;
    }
  }
};

// broadcast lane 0's list state to the wave (only lane 0 mutates L)
__device__ __forceinline__ void seg_bcast(SegList& L) {
  L.n = __shfl(L.n, 0, 64);
  L.prun = __shfl(L.prun, 0, 64);
  L.overflow = __shfl(L.overflow, 0, 64);
}

// Walk every valid element of a summary's run after its first one (first, end)
// as a single-element piece (exact fallback for a summary whose segments
// overflowed).  Whole wave: 64 elements per step are loaded in parallel; a step
// without a new prefix-max record merges with two wave reductions, otherwise
// lane 0 walks it from LDS.  L must be wave-uniform on entry and is on exit.
__device__ void rewalk_piece(const RankQ& Q, int32_t first, int32_t end, SegList& L, int32_t* sP, int32_t* sO) {
  const int lane = threadIdx.x;
  for (int64_t b = (int64_t)first + 1; b < end; b += 64) {
    const int64_t e = b + lane;
    bool ok = e < end && !(Q.removed && ldg(Q.removed + e));
    int32_t p = -1, od = 0;
    if (ok) {
      p = (int32_t)(ldg(Q.feat + e * FEAT_WORDS) & 0xFFFF);
      od = (int32_t)((ldg(Q.feat + e * FEAT_WORDS + 1) >> 16) & 0xFF);
    }
    if (__all(!ok || p <= L.prun)) {
      const int32_t m = wave_max_i(ok ? od : 0);
      const int32_t key = wave_max_i((ok && od > 0) ? ((lane + 1) << 8) | od : 0);
      if (lane == 0 && (m > 0 || key > 0)) L.add(-1, m, key & 0xFF);
    } else {
      sP[lane] = ok ? p : -2;
      sO[lane] = od;
      __syncthreads();
      if (lane == 0)
        for (int i = 0; i < 64; i++)
          if (sP[i] != -2) L.add(sP[i], sO[i], sO[i]);
      __syncthreads();
    }
    seg_bcast(L);
  }
}

// what the ordered fold reads of one chunk summary (nvc 0: empty or past the end)
struct FoldIn {
  int32_t nvc, pm, Mall, Lall, pf, of, ns, first, end;
};
__device__ __forceinline__ FoldIn fold_in(const ChunkSum* C, int64_t c, int64_t nc) {
  FoldIn f{0, -1, 0, 0, 0, 0, 0, 0, 0};
  if (c < nc) {
    const ChunkSum& X = C[c];
    f.nvc = X.nvalid;
    f.pm = X.pmax;
    f.Mall = max(X.od_first, X.M_rest);
    f.Lall = X.L_rest > 0 ? X.L_rest : (X.od_first > 0 ? X.od_first : 0);
    f.pf = X.p_first;
    f.of = X.od_first;
    f.ns = X.overflow ? -1 : X.nseg;
    f.first = X.first;
    f.end = X.end;
  }
  return f;
}

// Authority host counts by partition (ReferenceOrder doms / maxdomcount,
// :176-216) for queries whose records carry dense host ids, on one context
// (RankQ::ecnt; sharded contexts keep the host tables the owner exchange reads).
// A query's valid elements are spread over hp_nb buckets by a hash of their host
// id (k_reduce counts per chunk and bucket as it streams the records -- round 5
// ran a separate k_hpart_hist pass over them, 6.5 us on C5 --, a scan gives every (bucket, chunk)
// its place, k_hpart_scatter writes (host id, element) there); every host lands in
// exactly one bucket, so one workgroup per bucket (k_hbucket) counts its hosts in
// LDS, writes every element's host count (ecnt, what cardinal reads) and folds
// the bucket's largest count into maxdomcount -- no global atomic per posting, no
// table probe per scored posting.  A bucket whose hosts overflow its LDS table
// counts the rest in the query's global host table (only its workgroup touches
// those hosts, so their counts are final when it reads them back).
__global__ __launch_bounds__(CHUNK_THREADS) void k_hpart_scatter(const RankQ* __restrict__ qs,
                                                                 const int32_t* __restrict__ chunk_q,
                                                                 const int32_t* __restrict__ hoffs,
                                                                 uint2* __restrict__ part) {
  __shared__ int32_t sC[HPART_MAXS];
  const int64_t b = blockIdx.x;
  const RankQ& Q = qs[chunk_q[b]];
  if (!Q.ecnt) return;
  const int64_t c = b - Q.chunk_base;
  const int nb = Q.hp_nb;
  for (int i = threadIdx.x; i < nb; i += CHUNK_THREADS) sC[i] = hoffs[Q.hp_hoff + (int64_t)i * Q.nchunks + c];
  __syncthreads();
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++) {
    const int64_t e = c * CHUNK + s * CHUNK_THREADS + threadIdx.x;
    if (e < Q.n && !(Q.removed && ldg(Q.removed + e))) {
      const uint32_t h = (uint32_t)(ldg(Q.feat + e * FEAT_WORDS + 3) >> 34);
      const int32_t pos = atomicAdd(&sC[hp_bucket(h, nb)], 1);
      part[pos] = make_uint2(h, (uint32_t)e);
    }
  }
}

__global__ __launch_bounds__(CHUNK_THREADS) void k_hbucket(const RankQ* __restrict__ qs, const int2* __restrict__ bq,
                                                           const int32_t* __restrict__ hoffs,
                                                           const uint2* __restrict__ part,
                                                           ShardSum* __restrict__ shard) {
  __shared__ uint32_t sK[HB_SLOTS];
  __shared__ uint32_t sN[HB_SLOTS];
  const int2 qb = bq[blockIdx.x];
  const RankQ& Q = qs[qb.x];
  const int64_t i0 = hoffs[Q.hp_hoff + (int64_t)qb.y * Q.nchunks];
  const int64_t i1 = hoffs[Q.hp_hoff + (int64_t)(qb.y + 1) * Q.nchunks];
  for (int i = threadIdx.x; i < HB_SLOTS; i += CHUNK_THREADS) sK[i] = sN[i] = 0;
  __syncthreads();
  // count: LDS table (key = host id + 1), the query's global table past 32 probes
  for (int64_t i = i0 + threadIdx.x; i < i1; i += CHUNK_THREADS) {
    const uint32_t key = ldg(&part[i].x) + 1u;
    uint32_t slot = (key * 0x9E3779B1u) >> (32 - HB_LOG2);
    bool done = false;
    for (int p = 0; p < 32 && !done; p++, slot = (slot + 1) & (HB_SLOTS - 1)) {
      const uint32_t prev = atomicCAS(&sK[slot], 0u, key);
      if (prev == 0u || prev == key) {
        atomicAdd(&sN[slot], 1u);
        done = true;
      }
    }
    if (!done) {
      uint64_t gs = mix64((uint64_t)key) & Q.hmask;
      while (true) {
        const unsigned long long prev = atomicCAS((unsigned long long*)&Q.hkeys[gs], 0ull, (unsigned long long)key);
        if (prev == 0ull || prev == (unsigned long long)key) {
          atomicAdd(&Q.hcnt[gs], 1u);
          break;
        }
        gs = (gs + 1) & Q.hmask;
      }
    }
  }
  __syncthreads();
  __threadfence_block();
  // every element's host count (what cardinal reads), the bucket's largest count
  int32_t hmax = 0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += CHUNK_THREADS) {
    const uint2 it = part[i];
    const uint32_t key = it.x + 1u;
    uint32_t slot = (key * 0x9E3779B1u) >> (32 - HB_LOG2);
    int32_t cnt = -1;
    for (int p = 0; p < 32; p++, slot = (slot + 1) & (HB_SLOTS - 1)) {
      const uint32_t k = sK[slot];
      if (k == key) { cnt = (int32_t)sN[slot]; break; }
      if (k == 0u) break;
    }
    if (cnt < 0) {  // counted in the global table: read it with atomics (this kernel wrote it)
      uint64_t gs = mix64((uint64_t)key) & Q.hmask;
      while (atomicAdd((unsigned long long*)&Q.hkeys[gs], 0ull) != (unsigned long long)key) gs = (gs + 1) & Q.hmask;
      cnt = (int32_t)atomicAdd(&Q.hcnt[gs], 0u);
    }
    stg(Q.ecnt + it.y, cnt);
    hmax = max(hmax, cnt);
  }
  const int32_t wm = wave_max_i(hmax);
  if ((threadIdx.x & 63) == 0 && wm > 0) atomicMax(&shard[qb.x].maxdom, wm);
}

// What an ordered combination of summaries yields besides its fold pieces.
struct FoldRes {
  int32_t nv, vamn, vamx;
  int64_t firstc;  // the first summary with a valid element
  int32_t mn[NF], mx[NF];
  double tfmn, tfmx;
};

// Ordered combination (one wave) of the summaries C[0, nc), in container order:
// the order-independent parts into R, the fold's pieces into L.
__device__ void fold_run(const RankQ& Q, const ChunkSum* __restrict__ C, int64_t nc, SegList& L, int32_t* sRw,
                         FoldRes& R) {
  const int lane = threadIdx.x;
  // ---- min / max / counts / first chunk, one pass.  virtualAge over the shard's
  // rest = chunk rests + first elements of every chunk but the shard's first: each
  // lane keeps its own first chunk's first element aside until the shard's first
  // chunk is known.
  int32_t mn[NF], mx[NF];
  for (int f = 0; f < NF; f++) { mn[f] = BIG; mx[f] = -1; }
  double tfmn = 1e300, tfmx = -1e300;
  int32_t nv = 0, vamn = BIG, vamx = -1, a_lane = -1;
  int64_t lanec = INT64_MAX;
  for (int64_t c = lane; c < nc; c += 64) {
    const ChunkSum& X = C[c];
    if (X.nvalid == 0) continue;
    nv += X.nvalid;
    for (int f = 0; f < NF; f++) { mn[f] = min(mn[f], X.mn[f]); mx[f] = max(mx[f], X.mx[f]); }
    tfmn = fmin(tfmn, X.tf_mn);
    tfmx = fmax(tfmx, X.tf_mx);
    vamn = min(vamn, X.va_mn_rest);
    vamx = max(vamx, X.va_mx_rest);
    if (lanec == INT64_MAX) {
      lanec = c;
      a_lane = X.a_first;
    } else {
      vamn = min(vamn, X.a_first);
      vamx = max(vamx, X.a_first);
    }
  }
  for (int f = 0; f < NF; f++) { mn[f] = wave_min_i(mn[f]); mx[f] = wave_max_i(mx[f]); }
  tfmn = wave_min_d(tfmn);
  tfmx = wave_max_d(tfmx);
  nv = wave_sum_i(nv);
  const int64_t firstc = wave_min_i((int32_t)(lanec == INT64_MAX ? BIG : lanec));
  if (lanec != INT64_MAX && lanec != firstc) { vamn = min(vamn, a_lane); vamx = max(vamx, a_lane); }
  vamn = wave_min_i(vamn);
  vamx = wave_max_i(vamx);

  // ---- ordered fold pieces
  if (nv > 0) {
    const ChunkSum& X = C[firstc];
    if (X.overflow) rewalk_piece(Q, X.first, X.end, L, sRw, sRw + 64);
    else if (lane == 0)
      for (int i = 0; i < X.nseg; i++) L.add((int32_t)(X.seg[i] >> 16), (int32_t)((X.seg[i] >> 8) & 0xFF), (int32_t)(X.seg[i] & 0xFF));
  }
  seg_bcast(L);
  // The later chunks, 64 at a time (lane i: chunk c0+i; the next batch is loaded
  // while this one is folded).  A chunk is a record chunk iff its max posintext
  // exceeds the running P before it (prefix max over the batch, seeded with
  // L.prun); only record chunks add pieces of their own.  The chunks between two
  // record chunks merge into the last piece as one (max od, last positive od),
  // taken by a segmented scan headed at the record lanes.
  const int64_t cs0 = nv > 0 ? firstc + 1 : nc;
  FoldIn cur = fold_in(C, cs0 + lane, nc);
  for (int64_t c0 = cs0; c0 < nc; c0 += 64) {
    const FoldIn nxt = fold_in(C, c0 + 64 + lane, nc);
    const int32_t pinc = wave_incl_max(cur.nvc ? cur.pm : -1);
    int32_t pex = __shfl_up(pinc, 1, 64);
    pex = max(lane == 0 ? -1 : pex, L.prun);
    const bool rec = cur.nvc && cur.pm > pex;
    const uint64_t heads = __ballot(rec);
    int32_t m = (cur.nvc && !rec) ? cur.Mall : 0;
    int32_t key = (cur.nvc && !rec && cur.Lall > 0) ? ((lane + 1) << 8) | cur.Lall : 0;
    bool hd = rec;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t m2 = __shfl_up(m, o, 64), k2 = __shfl_up(key, o, 64);
      const bool h2 = __shfl_up((int)hd, o, 64) != 0;
      if (lane >= o && !hd) { m = max(m, m2); key = max(key, k2); hd = h2; }
    }
    // run before the first record chunk
    const int pre_end = heads ? __ffsll((long long)heads) - 2 : 63;
    if (pre_end >= 0) {
      const int32_t em = __shfl(m, pre_end, 64), ek = __shfl(key, pre_end, 64);
      if (lane == 0 && (em > 0 || ek > 0)) L.add(-1, em, ek & 0xFF);
    }
    uint64_t hm = heads;
    while (hm) {  // wave-uniform
      const int r = __ffsll((long long)hm) - 1;
      hm &= hm - 1;
      const int end = hm ? __ffsll((long long)hm) - 2 : 63;
      const int32_t pf = __shfl(cur.pf, r, 64), of = __shfl(cur.of, r, 64);
      const int32_t ns = __shfl(cur.ns, r, 64), fi = __shfl(cur.first, r, 64), en = __shfl(cur.end, r, 64);
      if (lane == 0) L.add(pf, of, of);
      if (ns < 0) {
        seg_bcast(L);
        rewalk_piece(Q, fi, en, L, sRw, sRw + 64);
      } else {
        const uint32_t sg = lane < ns ? C[c0 + r].seg[lane] : 0u;
        for (int s = 0; s < ns; s++) {
          const uint32_t v = __shfl(sg, s, 64);
          if (lane == 0) L.add((int32_t)(v >> 16), (int32_t)((v >> 8) & 0xFF), (int32_t)(v & 0xFF));
        }
      }
      const int32_t em = __shfl(m, end, 64), ek = __shfl(key, end, 64);
      if (lane == 0 && (em > 0 || ek > 0)) L.add(-1, em, ek & 0xFF);
      seg_bcast(L);
    }
    seg_bcast(L);
    cur = nxt;
  }
  R.nv = nv;
  R.vamn = vamn;
  R.vamx = vamx;
  R.firstc = firstc;
  for (int f = 0; f < NF; f++) { R.mn[f] = mn[f]; R.mx[f] = mx[f]; }
  R.tfmn = tfmn;
  R.tfmx = tfmx;
}

// one wave per query: ordered combination of the summaries of this shard -- the
// chunk summaries of k_reduce, or the merged compaction pieces (RankQ::groups)
__global__ __launch_bounds__(64) void k_shard_fin(const RankQ* __restrict__ qs, const int64_t* __restrict__ chunk_base,
                                                  const ChunkSum* __restrict__ cs, ShardSum* __restrict__ out) {
  __shared__ uint32_t sSeg[SSEG];
  __shared__ int32_t sRw[128];
  const int qi = blockIdx.x;
  const RankQ& Q = qs[qi];
  const int lane = threadIdx.x;
  const ChunkSum* C = Q.pieces ? Q.groups : cs + chunk_base[qi];
  const int64_t nc = Q.pieces ? Q.ngroups : Q.nchunks;
  ShardSum& S = out[qi];
  if (!Q.pieces && nc == 1 && !C[0].overflow) return;  // k_reduce wrote this one (one chunk, no overflow)
  SegList L{sSeg, SSEG, 0, 0, -1};
  FoldRes R;
  fold_run(Q, C, nc, L, sRw, R);
  __syncthreads();
  if (lane == 0) {
    S.nvalid = R.nv;
    S.has_first = R.nv > 0;
    if (R.nv > 0) {
      S.p_first = C[R.firstc].p_first;
      S.od_first = C[R.firstc].od_first;
      S.a_first = C[R.firstc].a_first;
    } else {
      S.p_first = S.od_first = S.a_first = 0;
    }
    for (int f = 0; f < NF; f++) { S.mn[f] = R.mn[f]; S.mx[f] = R.mx[f]; }
    S.va_mn_rest = R.vamn;
    S.va_mx_rest = R.vamx;
    S.tf_mn = R.tfmn;
    S.tf_mx = R.tfmx;
    S.nseg = L.n > SSEG ? SSEG : L.n;
    S.overflow = L.overflow;
  }
  for (int i = lane; i < SSEG && i < L.n; i += 64) S.seg[i] = sSeg[i];
}

// The compaction's tile pieces of a query (RankQ::pieces) merged 64 at a time into
// one ChunkSum each (RankQ::groups), one wave per group, all groups of the batch
// at once: k_shard_fin then folds a few summaries per query, as many as k_reduce
// would have written for its chunks, instead of every tile's in one wave.
__global__ __launch_bounds__(64) void k_piece_merge(const RankQ* __restrict__ qs, const int2* __restrict__ group_q) {
  __shared__ uint32_t sSeg[SEGC];
  __shared__ int32_t sRw[128];
  const int2 gq = group_q[blockIdx.x];  // (query, group)
  const RankQ& Q = qs[gq.x];
  const int lane = threadIdx.x;
  const int64_t c0 = (int64_t)gq.y * 64;
  const ChunkSum* C = Q.pieces + c0;
  const int64_t nc = min((int64_t)64, Q.npieces - c0);
  ChunkSum& S = Q.groups[gq.y];
  SegList L{sSeg, SEGC, 0, 0, -1};
  FoldRes R;
  fold_run(Q, C, nc, L, sRw, R);
  // pmax over every element; over the rest: max stored distance (the first
  // summary's rest, every later summary whole) and the last positive one
  const FoldIn f = fold_in(C, lane, nc);
  const int32_t fc = (int32_t)R.firstc;
  const int32_t pm = wave_max_i(f.nvc ? f.pm : -1);
  const int32_t mr = wave_max_i(!f.nvc ? 0 : lane == fc ? C[lane].M_rest : lane > fc ? f.Mall : 0);
  const int32_t lk = wave_max_i(f.nvc && lane > fc && f.Lall > 0 ? ((lane + 1) << 8) | f.Lall : 0);
  __syncthreads();
  if (lane == 0) {
    S.nvalid = R.nv;
    S.end = nc > 0 ? C[nc - 1].end : 0;
    if (R.nv > 0) {
      const ChunkSum& F = C[fc];
      S.first = F.first;
      S.p_first = F.p_first;
      S.od_first = F.od_first;
      S.a_first = F.a_first;
      S.L_rest = lk ? (lk & 0xFF) : F.L_rest;
    } else {
      S.first = -1;
      S.p_first = S.od_first = S.a_first = 0;
      S.L_rest = 0;
    }
    S.pmax = pm;
    S.M_rest = mr;
    for (int k = 0; k < NF; k++) { S.mn[k] = R.mn[k]; S.mx[k] = R.mx[k]; }
    S.va_mn_rest = R.vamn;
    S.va_mx_rest = R.vamx;
    S.tf_mn = R.tfmn;
    S.tf_mx = R.tfmx;
    S.nseg = L.n;
    S.overflow = L.overflow;
  }
  if (lane < SEGC && lane < L.n) S.seg[lane] = sSeg[lane];
}

// fold state transition for one piece (WordReferenceVars.max :431-445)
struct Fold {
  int32_t P, A;
  bool hasA;
  __device__ void piece(int32_t Pj, int32_t M, int32_t Lp) {
    int32_t Pe = max(P, Pj);
    if (Pe > 0) {
      int32_t d0 = hasA ? abs(Pe - A) : 0;
      if (M > d0) { A = Pe + M; hasA = true; }
    } else if (Lp > 0) {
      A = Lp;
      hasA = true;
    }
    P = Pe;
  }
  __device__ int32_t D() const { return (hasA && P > 0) ? abs(P - A) : 0; }
};

// one thread per query: combine `world` shard summaries in shard (= url-hash) order
__global__ void k_combine(const RankQ* __restrict__ qs, int nq, const ShardSum* __restrict__ sh, int world,
                          NormState* __restrict__ norm) {
  const int qi = blockIdx.x * blockDim.x + threadIdx.x;
  if (qi >= nq) return;
  const RankQ& Q = qs[qi];
  NormState N;
  for (int f = 0; f < NF; f++) { N.mn[f] = BIG; N.mx[f] = -1; }
  N.tf_mn = 1e300;
  N.tf_mx = -1e300;
  N.va_mn = BIG;
  N.va_mx = -1;
  N.nvalid = 0;
  N.maxdom = 0;
  int gf = -1, ovf = 0;
  for (int s = 0; s < world; s++) {
    const ShardSum& X = sh[(int64_t)s * nq + qi];
    if (X.nvalid == 0) continue;
    if (gf < 0) gf = s;
    N.nvalid += X.nvalid;
    for (int f = 0; f < NF; f++) { N.mn[f] = min(N.mn[f], X.mn[f]); N.mx[f] = max(N.mx[f], X.mx[f]); }
    N.tf_mn = fmin(N.tf_mn, X.tf_mn);
    N.tf_mx = fmax(N.tf_mx, X.tf_mx);
    // the very first element is min/max's clone: its virtualAge is clamped (:357-361)
    int32_t af = (s == gf) ? clamp_days(X.a_first, Q.now_ms) : X.a_first;
    N.va_mn = min(N.va_mn, min(af, X.va_mn_rest));
    N.va_mx = max(N.va_mx, max(af, X.va_mx_rest));
    N.maxdom = max(N.maxdom, X.maxdom);
    ovf |= X.overflow;
  }
  Fold fd{0, 0, false};
  if (gf >= 0) {
    if (ovf && world == 1) {
      // exact sequential fold over the whole container
      bool first = true;
      for (int64_t e = 0; e < Q.n; e++) {
        if (Q.removed && ldg(Q.removed + e)) continue;
        int32_t p = (int32_t)(ldg(Q.feat + e * FEAT_WORDS) & 0xFFFF);
        int32_t od = (int32_t)((ldg(Q.feat + e * FEAT_WORDS + 1) >> 16) & 0xFF);
        if (first) { fd.P = p; first = false; }
        else fd.piece(p, od, od);
      }
    } else {
      for (int s = gf; s < world; s++) {
        const ShardSum& X = sh[(int64_t)s * nq + qi];
        if (X.nvalid == 0) continue;
        if (s == gf) fd.P = X.p_first;
        else fd.piece(X.p_first, X.od_first, X.od_first);
        for (int i = 0; i < X.nseg; i++)
          fd.piece((int32_t)(X.seg[i] >> 16), (int32_t)((X.seg[i] >> 8) & 0xFF), (int32_t)(X.seg[i] & 0xFF));
      }
    }
  }
  N.D = (ovf && world > 1) ? -1 : fd.D();
  if (N.nvalid == 0) {
    for (int f = 0; f < NF; f++) { N.mn[f] = 0; N.mx[f] = 0; }
    N.va_mn = N.va_mx = 0;
    N.tf_mn = N.tf_mx = 0.0;
  }
  for (int f = 0; f < NF; f++) N.rcp[f] = N.mx[f] != N.mn[f] ? 1.0 / (double)(N.mx[f] - N.mn[f]) : 0.0;
  N.rcp[NF] = N.va_mx != N.va_mn ? 1.0 / (double)(N.va_mx - N.va_mn) : 0.0;
  N.rcp[NF + 1] = N.D != 0 ? 1.0 / (double)N.D : 0.0;
  norm[qi] = N;
}

// ------------------------------------------------------------------ scoring
// Java int division n / d (truncation toward zero) for |n| < 2^24 and
// 0 < d < 2^24, with r = fl(1/d): |n|*r carries an error below 2^-28 and the
// 2^-26 bias lifts exact quotients above their integer while a true fraction
// (at least 1/d > 2^-24 below the next integer) stays below it, so the
// truncation equals the integer quotient.  Every normalised term of cardinal
// has |(t - min) << 8| <= 65535 * 256 < 2^24 and max - min <= 65535.
__device__ __forceinline__ int32_t qdiv(int32_t n, double r) {
  const int32_t q = (int32_t)fma((double)(n < 0 ? -n : n), r, 0x1p-26);
  return n < 0 ? -q : q;
}

// The long-accumulated flag and language terms of cardinal (ReferenceOrder.java:242-260)
// added to R; Bitfield bit j is bit j of z (Bitfield.java:88-93, Tokenizer.java:51-56).
__device__ __forceinline__ int64_t flags_lang_terms(int64_t R, uint32_t z, uint32_t lang, const RankQ& Q) {
  const yrwi_profile& rk = Q.prof;
  const int32_t c255 = 255;
  if (z & (1u << 28)) R = add64(R, shl32(c255, rk.coeff_appurl));
  if (z & (1u << 25)) R = add64(R, shl32(c255, rk.coeff_app_dc_title));
  if (z & (1u << 26)) R = add64(R, shl32(c255, rk.coeff_app_dc_creator));
  if (z & (1u << 27)) R = add64(R, shl32(c255, rk.coeff_app_dc_subject));
  if (z & (1u << 24)) R = add64(R, shl32(c255, rk.coeff_app_dc_description));
  if (z & (1u << 29)) R = add64(R, shl32(c255, rk.coeff_appemph));
  if (z & (1u << 0)) R = add64(R, shl32(c255, rk.coeff_catindexof));
  if (z & (1u << 20)) R = add64(R, shl32(c255, rk.coeff_cathasimage));
  if (z & (1u << 21)) R = add64(R, shl32(c255, rk.coeff_cathasaudio));
  if (z & (1u << 22)) R = add64(R, shl32(c255, rk.coeff_cathasvideo));
  if (z & (1u << 23)) R = add64(R, shl32(c255, rk.coeff_cathasapp));
  if (Q.lang_ok && lang == ((uint32_t)Q.lang[0] | ((uint32_t)Q.lang[1] << 8))) R = add64(R, shl32(c255, rk.coeff_language));
  return R;
}

// Normalised int terms of cardinal (ReferenceOrder.java:223-241): inv counts
// "smaller is better" fields, fwd "larger is better"; 0 where max == min.
__device__ __forceinline__ int32_t term_inv(int32_t tv, int32_t lo, int32_t hi, double rc, int32_t c) {
  if (hi == lo) return 0;
  return shl32(sub32(256, qdiv(shl32(sub32(tv, lo), 8), rc)), c);
}
__device__ __forceinline__ int32_t term_fwd(int32_t tv, int32_t lo, int32_t hi, double rc, int32_t c) {
  if (hi == lo) return 0;
  return shl32(qdiv(shl32(sub32(tv, lo), 8), rc), c);
}

// Per-query term tables (in LDS), built by every scoring workgroup:
//  t    the nine one-byte fields' terms, CARD_TABS x 256 int32: a term depends on
//       the field value alone, and int addition wraps associatively, so summing
//       looked-up terms equals cardinal's running int sum;
//  flo  the long sum of the flag terms of Bitfield bits 20-23 for each subset,
//  fhi  the same for bits 24-29 (the flag terms are independent long additions).
constexpr int CARD_TABS = 9;
enum : int { CT_URLCOMPS = 0, CT_URLLENGTH, CT_POSOFPHRASE, CT_POSINPHRASE, CT_DISTANCE, CT_WORDSINTITLE,
             CT_LLOCAL, CT_LOTHER, CT_HITCOUNT };
struct CardTab {
  int32_t t[CARD_TABS * 256];
  int64_t flo[16];
  int64_t fhi[64];
};
__device__ __forceinline__ void build_card_tab(CardTab* T, const NormState& N, const RankQ& Q) {
  const yrwi_profile& rk = Q.prof;
  for (int i = threadIdx.x; i < CARD_TABS * 256; i += blockDim.x) {
    const int v = i & 255;
    int32_t r;
    switch (i >> 8) {
      case CT_URLCOMPS:
        r = term_inv(v, N.mn[F_URLCOMPS], N.mx[F_URLCOMPS], N.rcp[F_URLCOMPS], rk.coeff_urlcomps);
        break;
      case CT_URLLENGTH:
        r = term_inv(v, N.mn[F_URLLENGTH], N.mx[F_URLLENGTH], N.rcp[F_URLLENGTH], rk.coeff_urllength);
        break;
      case CT_POSOFPHRASE:
        r = term_inv(v, N.mn[F_POSOFPHRASE], N.mx[F_POSOFPHRASE], N.rcp[F_POSOFPHRASE], rk.coeff_posofphrase);
        break;
      case CT_POSINPHRASE:
        r = term_inv(v, N.mn[F_POSINPHRASE], N.mx[F_POSINPHRASE], N.rcp[F_POSINPHRASE], rk.coeff_posinphrase);
        break;
      case CT_DISTANCE: r = term_inv(v, 0, N.D, N.rcp[NF + 1], rk.coeff_worddistance); break;
      case CT_WORDSINTITLE:
        r = term_fwd(v, N.mn[F_WORDSINTITLE], N.mx[F_WORDSINTITLE], N.rcp[F_WORDSINTITLE], rk.coeff_wordsintitle);
        break;
      case CT_LLOCAL: r = term_fwd(v, N.mn[F_LLOCAL], N.mx[F_LLOCAL], N.rcp[F_LLOCAL], rk.coeff_llocal); break;
      case CT_LOTHER: r = term_fwd(v, N.mn[F_LOTHER], N.mx[F_LOTHER], N.rcp[F_LOTHER], rk.coeff_lother); break;
      default: r = term_fwd(v, N.mn[F_HITCOUNT], N.mx[F_HITCOUNT], N.rcp[F_HITCOUNT], rk.coeff_hitcount); break;
    }
    T->t[i] = r;
  }
  const int i = threadIdx.x;
  if (i < 16) T->flo[i] = flags_lang_terms(0, (uint32_t)i << 20, ~0u, Q) - flags_lang_terms(0, 0, ~0u, Q);
  else if (i < 80) T->fhi[i - 16] = flags_lang_terms(0, (uint32_t)(i - 16) << 24, ~0u, Q) - flags_lang_terms(0, 0, ~0u, Q);
}
// flags_lang_terms through the tables
__device__ __forceinline__ int64_t flags_lang_tab(int64_t R, uint32_t z, uint32_t lang, const RankQ& Q,
                                                  const CardTab* T) {
  const yrwi_profile& rk = Q.prof;
  R = add64(R, T->flo[(z >> 20) & 15u]);
  R = add64(R, T->fhi[(z >> 24) & 63u]);
  if (z & 1u) R = add64(R, shl32(255, rk.coeff_catindexof));
  if (Q.lang_ok && lang == ((uint32_t)Q.lang[0] | ((uint32_t)Q.lang[1] << 8))) R = add64(R, shl32(255, rk.coeff_language));
  return R;
}

// ReferenceOrder.cardinal(WordReference) (ReferenceOrder.java:223-265), settled
// min/max; with tab (build_card_tab) the one-byte fields' terms are looked up.
__device__ __forceinline__ int64_t cardinal(const Feat& t, const NormState& N, const RankQ& Q, int32_t hcount,
                                            const CardTab* tab = nullptr) {
  const yrwi_profile& rk = Q.prof;
  int32_t tfterm = 0;
  if (!(N.tf_mx == N.tf_mn))
    tfterm = shl32(d2i(((t.tf - N.tf_mn) * 256.0) / (N.tf_mx - N.tf_mn)), rk.coeff_termfrequency);
  const int dl = t.dl;  // DigestURL.domLengthEstimation; << (8/20) == << 0
  const int32_t dln = dl == 0 ? 4 : dl == 1 ? 10 : dl == 2 ? 14 : 20;
  int32_t s = shl32(256 - dln, rk.coeff_domlength);
  if (tab) {
    s = add32(s, tab->t[CT_URLCOMPS * 256 + t.f[F_URLCOMPS]]);
    s = add32(s, tab->t[CT_URLLENGTH * 256 + t.f[F_URLLENGTH]]);
    s = add32(s, tab->t[CT_POSOFPHRASE * 256 + t.f[F_POSOFPHRASE]]);
    s = add32(s, tab->t[CT_POSINPHRASE * 256 + t.f[F_POSINPHRASE]]);
    s = add32(s, tab->t[CT_DISTANCE * 256 + t.od]);
    s = add32(s, tab->t[CT_WORDSINTITLE * 256 + t.f[F_WORDSINTITLE]]);
    s = add32(s, tab->t[CT_LLOCAL * 256 + t.f[F_LLOCAL]]);
    s = add32(s, tab->t[CT_LOTHER * 256 + t.f[F_LOTHER]]);
    s = add32(s, tab->t[CT_HITCOUNT * 256 + t.f[F_HITCOUNT]]);
  } else {
    s = add32(s, term_inv(t.f[F_URLCOMPS], N.mn[F_URLCOMPS], N.mx[F_URLCOMPS], N.rcp[F_URLCOMPS], rk.coeff_urlcomps));
    s = add32(s, term_inv(t.f[F_URLLENGTH], N.mn[F_URLLENGTH], N.mx[F_URLLENGTH], N.rcp[F_URLLENGTH],
                          rk.coeff_urllength));
    s = add32(s, term_inv(t.f[F_POSOFPHRASE], N.mn[F_POSOFPHRASE], N.mx[F_POSOFPHRASE], N.rcp[F_POSOFPHRASE],
                          rk.coeff_posofphrase));
    s = add32(s, term_inv(t.f[F_POSINPHRASE], N.mn[F_POSINPHRASE], N.mx[F_POSINPHRASE], N.rcp[F_POSINPHRASE],
                          rk.coeff_posinphrase));
    s = add32(s, term_inv(t.od, 0, N.D, N.rcp[NF + 1], rk.coeff_worddistance));
    s = add32(s, term_fwd(t.f[F_WORDSINTITLE], N.mn[F_WORDSINTITLE], N.mx[F_WORDSINTITLE], N.rcp[F_WORDSINTITLE],
                          rk.coeff_wordsintitle));
    s = add32(s, term_fwd(t.f[F_LLOCAL], N.mn[F_LLOCAL], N.mx[F_LLOCAL], N.rcp[F_LLOCAL], rk.coeff_llocal));
    s = add32(s, term_fwd(t.f[F_LOTHER], N.mn[F_LOTHER], N.mx[F_LOTHER], N.rcp[F_LOTHER], rk.coeff_lother));
    s = add32(s, term_fwd(t.f[F_HITCOUNT], N.mn[F_HITCOUNT], N.mx[F_HITCOUNT], N.rcp[F_HITCOUNT], rk.coeff_hitcount));
  }
  s = add32(s, term_inv(t.f[F_POSINTEXT], N.mn[F_POSINTEXT], N.mx[F_POSINTEXT], N.rcp[F_POSINTEXT], rk.coeff_posintext));
  s = add32(s, term_fwd(t.a, N.va_mn, N.va_mx, N.rcp[NF], rk.coeff_date));
  s = add32(s, term_fwd(t.f[F_WORDSINTEXT], N.mn[F_WORDSINTEXT], N.mx[F_WORDSINTEXT], N.rcp[F_WORDSINTEXT],
                        rk.coeff_wordsintext));
  s = add32(s, term_fwd(t.f[F_PHRASESINTEXT], N.mn[F_PHRASESINTEXT], N.mx[F_PHRASESINTEXT], N.rcp[F_PHRASESINTEXT],
                        rk.coeff_phrasesintext));
  int64_t R = add64((int64_t)s, (int64_t)tfterm);  // + tf turns the sum into a long
  if (rk.coeff_authority > 12) {
    int32_t auth = div32(shl32(hcount, 8), add32(1, N.maxdom));  // ReferenceOrder.authority :213-216
    R = add64(R, (int64_t)shl32(auth, rk.coeff_authority));
  }
  return tab ? flags_lang_tab(R, t.z, t.lang, Q, tab) : flags_lang_terms(R, t.z, t.lang, Q);
}

__device__ __forceinline__ int32_t url_hashcode(const Row& r) {
  int32_t h = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) h = add32(mul32(31, h), (int32_t)r.b(j));
  return h;
}

__device__ __forceinline__ int32_t host_count(const RankQ& Q, uint64_t host) {
  uint64_t key = host + 1;
  uint64_t slot = mix64(key) & Q.hmask;
  while (true) {
    uint64_t k = Q.hkeys[slot];
    if (k == key) return (int32_t)Q.hcnt[slot];
    if (k == 0) return 0;
    slot = (slot + 1) & Q.hmask;
  }
}

// bitonic sort, descending on (k1, k2), N (power of two) entries in LDS, all NT threads participate
template <int NT>
__device__ __forceinline__ void bitonic_desc(uint64_t* k1, uint64_t* k2, int N) {
  for (int size = 2; size <= N; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < N / 2; i += NT) {
        const int pos = 2 * i - (i & (stride - 1));
        const int par = pos + stride;
        const bool desc = (pos & size) == 0;
        uint64_t a1 = k1[pos], a2 = k2[pos], b1 = k1[par], b2 = k2[par];
        const bool a_lt_b = a1 < b1 || (a1 == b1 && a2 < b2);
        if (a_lt_b == desc) {
          k1[pos] = b1; k2[pos] = b2;
          k1[par] = a1; k2[par] = a2;
        }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ int pow2_at_least(int n) {
  int p = 2;
  while (p < n) p <<= 1;
  return p;
}

// block exclusive scan (sum) for NT threads (multiple of 64, <= 1024); sh >= NT/64 ints
template <int NT>
__device__ __forceinline__ int32_t block_excl_sum(int32_t v, int32_t* sh, int32_t* tot) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int32_t inc = wave_incl_sum(v);
  if (lane == 63) sh[wv] = inc;
  __syncthreads();
  int32_t o = 0, all = 0;
  for (int w = 0; w < NT / 64; w++) { if (w < wv) o += sh[w]; all += sh[w]; }
  __syncthreads();
  *tot = all;
  return o + inc - v;
}

// dedupe (equal score and hashCode: the TreeSet keeps the first arrival) and
// compact the first `k` survivors of a sorted LDS list of N entries into out;
// returns the number written, *distinct = survivors before the cut at k
template <int NT>
__device__ __forceinline__ int32_t dedupe_take(const uint64_t* k1, const uint64_t* k2, int N, int32_t k, Cand* out,
                                               int32_t* sScan, int32_t* distinct,
                                               unsigned long long* publish = nullptr) {
  const int ipt = (N + NT - 1) / NT;  // <= 32
  const int i0 = threadIdx.x * ipt;
  int32_t keep = 0;
  uint32_t bits = 0;
  for (int s = 0; s < ipt; s++) {
    const int i = i0 + s;
    if (i >= N) break;
    bool v = k2[i] != 0;
    if (v && i > 0 && k1[i] == k1[i - 1] && (k2[i] >> 32) == (k2[i - 1] >> 32)) v = false;
    if (v) { bits |= 1u << s; keep++; }
  }
  int32_t tot;
  int32_t off = block_excl_sum<NT>(keep, sScan, &tot);
  for (int s = 0; s < ipt; s++) {
    if (bits & (1u << s)) {
      if (off < k) { out[off].k1 = k1[i0 + s]; out[off].k2 = k2[i0 + s]; }
      if (off == k - 1 && publish) atomicMax(publish, (unsigned long long)k1[i0 + s]);  // the k-th distinct class
      off++;
    }
  }
  if (distinct) *distinct = tot;
  return tot < k ? tot : k;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const uint64_t t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
  return v;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const uint64_t t = __shfl_xor(v, o, 64); v = t < v ? t : v; }
  return v;
}

// Radix-select digit search by one wave over a 256-bin histogram (descending
// digits): the bin holding the rem-th largest key -> sSel[0] = digit, sSel[1] =
// rank inside that bin, sSel[2] = keys in that bin.
__device__ __forceinline__ void radix_pick(const int32_t* sHist, int32_t rem, int32_t* sSel) {
  const int lane = threadIdx.x & 63;
  int32_t h4[4];
  int32_t sum = 0;
  for (int j = 0; j < 4; j++) { h4[j] = sHist[4 * lane + j]; sum += h4[j]; }
  const int32_t inc = wave_incl_sum(sum);
  const int32_t all = __shfl(inc, 63, 64);
  int32_t cum = all - inc;  // keys in higher bins than this lane's
  for (int j = 3; j >= 0; j--) {
    if (cum < rem && cum + h4[j] >= rem) { sSel[0] = 4 * lane + j; sSel[1] = rem - cum; sSel[2] = h4[j]; }
    cum += h4[j];
  }
}

// Per chunk: cardinal of every live posting, then the chunk's first kq distinct
// (score, hashCode) classes in TreeSet order.  The kq-th largest score key T is
// found by an MSB-first radix select (8-bit digits over the bits where the
// chunk's keys differ, LDS histograms); only keys >= T -- a prefix of the sorted
// chunk -- are sorted.  If the TreeSet dedupe leaves fewer than kq classes in
// that prefix, the whole chunk is sorted instead (exact either way).
// ------------------------------------------------ addRWIs constraints (filter)
// SearchEvent.addRWIs pollloop (SearchEvent.java:736-806) for one posting:
// doublecheck, flag counts, testFlags (:2459-2474), contentdom (Tokenizer flags
// :51-56, Response.DT_*), modifier.language, sitehash / siteexcludes.
__device__ __forceinline__ bool sorted_has_u64(const uint64_t* __restrict__ a, int64_t n, uint64_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo < n && a[lo] == x;
}

__device__ __forceinline__ bool flag_bit(uint32_t z, int j) { return (z >> j) & 1u; }  // Bitfield.get :88-93

__device__ __forceinline__ bool passes(const FilterQ& F, const Feat& t, uint64_t host);

// returns true if the posting enters the stack; counts flags into sFlag (LDS) when asked
// (hi, lo: the posting's url-hash key)
__device__ __forceinline__ bool admit(const FilterQ& F, const Feat& t, uint64_t hi, uint32_t lo, int32_t* sFlag) {
  if (F.nurl) {  // doublecheck: url already in SearchEvent.urlhashes
    int64_t a = 0, b = F.nurl;
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      const uint64_t mh = F.url_hi[m];
      if (mh < hi || (mh == hi && (uint32_t)F.url_lo[m] < lo)) a = m + 1; else b = m;
    }
    if (a < F.nurl && F.url_hi[a] == hi && (uint32_t)F.url_lo[a] == lo) return false;
  }
  if (sFlag)
    for (uint32_t m = t.z; m; m &= m - 1) atomicAdd(&sFlag[__ffs(m) - 1], 1);
  return passes(F, t, key_host36(hi, lo));
}

// the constraints after the doublecheck and the flag counts (:749-802); host =
// the posting's host hash (url-hash chars 6..11 as 36 bits)
__device__ __forceinline__ bool passes(const FilterQ& F, const Feat& t, uint64_t host) {
  const uint32_t z = t.z;
  if (F.has_constraint) {
    bool ok = F.all_of ? true : false;
    for (int j = 0; j < 32; j++) {
      const bool c = (F.constraint[j >> 3] >> (j & 7)) & 1u;
      if (!c) continue;
      if (F.all_of) { if (!flag_bit(z, j)) { ok = false; break; } }
      else if (flag_bit(z, j)) { ok = true; break; }
    }
    if (!ok) return false;
  }
  if (F.contentdom > 0) {
    const uint32_t d = t.d;
    bool bad;
    if (F.strict)
      bad = (F.contentdom == 2 && d != 'a') || (F.contentdom == 3 && d != 'm') || (F.contentdom == 1 && d != 'i') ||
            (F.contentdom == 4 && !flag_bit(z, 23));
    else
      bad = (F.contentdom == 2 && !flag_bit(z, 21)) || (F.contentdom == 3 && !flag_bit(z, 22)) ||
            (F.contentdom == 1 && !flag_bit(z, 20)) || (F.contentdom == 4 && !flag_bit(z, 23));
    if (bad) return false;
  }
  if (F.lang_len > 0) {  // modifier.language.equals(getLanguageString()): a 2-char string
    if (F.lang_len != 2 || (t.lang & 0xFFu) != F.lang[0] || (t.lang >> 8) != F.lang[1]) return false;
  }
  if (!F.has_site) {
    if (F.nsiteex && sorted_has_u64(F.siteex, F.nsiteex, host)) return false;
  } else if (host != F.site && (!F.has_alt || host != F.altsite)) {
    return false;
  }
  return true;
}

// Chunk scoring, two kernels.  k_score (small LDS footprint, so many chunks are
// resident per CU) handles every chunk whose selected prefix fits SCORE_SMALL
// entries and survives the TreeSet dedupe with kq classes -- all but chunks with
// long runs of tied scores or hashCode collisions; it appends the others to a
// redo list.  k_score_full re-scores those with the whole chunk in LDS.  Flag
// counts are taken once, by k_score.
constexpr int SCORE_SMALL = 256;
#ifndef YRWI_SCORE_CAP
#define YRWI_SCORE_CAP 128
#endif
constexpr int SCORE_CAP = YRWI_SCORE_CAP;  // early-exit bound of k_score's radix select (0: exact kq-th key)
static_assert(SCORE_CAP <= SCORE_SMALL, "the selected prefix must fit k_score's LDS");

// ---- per-query score threshold (k_score)
// A chunk that finds k distinct (score, hashCode) classes publishes the score of
// its k-th, s_c: at least k distinct classes of the query score >= s_c, so the
// query's k-th class does too, and no posting scoring below s_c can be among its
// top-k.  Later chunks of the query drop such postings before selection; with a
// cheap exact upper bound of a posting's score they skip its cardinal altogether.
//   bound = the int-summed terms' maxima (each normalised term <= 256 << c) except
//           domlength and date, computed exactly, + tf and authority maxima + the
//           exact flag / language terms
// valid while the int sum of terms 1-14 cannot wrap (PruneP.ok; else only the
// computed scores are compared with the threshold).
struct PruneP {
  int64_t hi32, lo32;  // sums of the bounded int terms' maxima / minima
  int64_t rest;        // tf and authority maxima (long-accumulated)
  int32_t ok;
};

__device__ __forceinline__ PruneP prune_params(const NormState& N, const RankQ& Q) {
  const yrwi_profile& rk = Q.prof;
  PruneP P{0, 0, 0, 1};
  auto term = [&](bool zero, int32_t c, int64_t vlo, int64_t vhi) {
    if (zero) return;
    const int64_t m = (int64_t)1 << (c & 31);
    const int64_t h = vhi * m, l = vlo * m;
    if (h >= ((int64_t)1 << 31) || l < -((int64_t)1 << 31)) P.ok = 0;  // the term itself could wrap
    P.hi32 += h;
    P.lo32 += l;
  };
  const int32_t* mn = N.mn;
  const int32_t* mx = N.mx;
  term(mx[F_URLCOMPS] == mn[F_URLCOMPS], rk.coeff_urlcomps, 0, 256);
  term(mx[F_URLLENGTH] == mn[F_URLLENGTH], rk.coeff_urllength, 0, 256);
  term(mx[F_POSINTEXT] == mn[F_POSINTEXT], rk.coeff_posintext, 0, 256);
  term(mx[F_POSOFPHRASE] == mn[F_POSOFPHRASE], rk.coeff_posofphrase, 0, 256);
  term(mx[F_POSINPHRASE] == mn[F_POSINPHRASE], rk.coeff_posinphrase, 0, 256);
  term(N.D == 0, rk.coeff_worddistance, 256 - 255 * 256, 256);  // stored distance up to 255 over D >= 1
  term(mx[F_WORDSINTITLE] == mn[F_WORDSINTITLE], rk.coeff_wordsintitle, 0, 256);
  term(mx[F_WORDSINTEXT] == mn[F_WORDSINTEXT], rk.coeff_wordsintext, 0, 256);
  term(mx[F_PHRASESINTEXT] == mn[F_PHRASESINTEXT], rk.coeff_phrasesintext, 0, 256);
  term(mx[F_LLOCAL] == mn[F_LLOCAL], rk.coeff_llocal, 0, 256);
  term(mx[F_LOTHER] == mn[F_LOTHER], rk.coeff_lother, 0, 256);
  term(mx[F_HITCOUNT] == mn[F_HITCOUNT], rk.coeff_hitcount, 0, 256);
  if (!(N.tf_mx == N.tf_mn)) {
    const int64_t h = (int64_t)256 << (rk.coeff_termfrequency & 31);
    if (h >= ((int64_t)1 << 31)) P.ok = 0;
    P.rest += h;
  }
  if (rk.coeff_authority > 12) {
    const int64_t h = (int64_t)255 << (rk.coeff_authority & 31);
    if (h >= ((int64_t)1 << 31)) P.ok = 0;
    P.rest += h;
  }
  return P;
}

// A query's pruning parameters and term tables, built once per query (k_qtabs,
// right before k_score) instead of in every chunk's workgroup: k_score's
// prologue took 5.2 of a C2 workgroup's 24.5 us (YRWI_PHASE_CLOCK), the dependent
// reads of the query's constants, thread 0's prune_params and the 2304-entry
// table build between two barriers; now one coalesced copy of 9.9 KB (L2-resident:
// every chunk of the query reads the same) beside the threshold's read.
struct QTab {
  PruneP P;
  CardTab T;
};
#ifndef YRWI_CARD_TAB_MIN
#define YRWI_CARD_TAB_MIN 512  // a chunk of at most this many postings computes its cardinals without the tables
#endif
__global__ __launch_bounds__(256) void k_qtabs(const RankQ* __restrict__ qs, const NormState* __restrict__ norm,
                                              QTab* __restrict__ out) {
  const int qi = blockIdx.x;
  const RankQ& Q = qs[qi];
  const NormState& N = norm[qi];
  if (Q.n > YRWI_CARD_TAB_MIN) build_card_tab(&out[qi].T, N, Q);  // (only chunks above it read the tables)
  if (threadIdx.x == 0) out[qi].P = prune_params(N, Q);
}
__device__ __forceinline__ void copy_card_tab(CardTab* dst, const CardTab* __restrict__ src) {
  static_assert(sizeof(CardTab) % 16 == 0, "16-B copies");
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  for (int i = threadIdx.x; i < (int)(sizeof(CardTab) / 16); i += blockDim.x) d4[i] = ldg(s4 + i);
}

// Upper bound of cardinal for a posting's record: domlength and date exactly
// (a posting's own date may lie above the clone-clamped maximum), the other
// int terms at their maxima, tf / authority maxima, flags and language exactly.
// *valid = 0 when the int sum of terms 1-14 could wrap for this posting (every
// partial sum lies in [exact + lo32, exact + hi32] since each term's range holds 0).
__device__ __forceinline__ int64_t score_bound(const Rec& q, const NormState& N, const RankQ& Q, const PruneP& P,
                                               bool* valid, const CardTab* tab = nullptr) {
  const yrwi_profile& rk = Q.prof;
  const int dl = (int)((q.w[3] >> 32) & 3);
  const int32_t dln = dl == 0 ? 4 : dl == 1 ? 10 : dl == 2 ? 14 : 20;
  int64_t ex = (int64_t)shl32(256 - dln, rk.coeff_domlength);
  if (N.va_mx != N.va_mn)
    ex += (int64_t)shl32(qdiv(shl32(sub32((int32_t)(q.w[2] & 0xFFFF), N.va_mn), 8), N.rcp[NF]), rk.coeff_date);
  *valid = P.ok && ex + P.hi32 < ((int64_t)1 << 31) && ex + P.lo32 >= -((int64_t)1 << 31);
  const uint32_t z = (uint32_t)(q.w[2] >> 32), lang = (uint32_t)((q.w[2] >> 16) & 0xFFFF);
  return tab ? flags_lang_tab(ex + P.hi32 + P.rest, z, lang, Q, tab) : flags_lang_terms(ex + P.hi32 + P.rest, z, lang, Q);
}

// score keys of one chunk: a[s] = score ^ 2^63 of element e0 + s*CHUNK_THREADS,
// bit s of the result set when that element is live and admitted (and, with a
// threshold T, its key >= T)
#ifdef YRWI_PHASE_CLOCK  // timing experiment only: per-block wall-clock stamps of k_score (thread 0)
constexpr int PH_MAXB = 16384;
__device__ unsigned long long g_ts[PH_MAXB * 8];
__device__ unsigned long long g_phase[16];
#define PHASE(i) \
  if (threadIdx.x == 0 && blockIdx.x < PH_MAXB) g_ts[blockIdx.x * 8 + 1 + (i)] = wall_clock64();
#else
#define PHASE(i)
#endif

// score keys of one chunk: a[s] = score ^ 2^63 of the chunk's element
// s*CHUNK_THREADS + tid (with idx: of element idx[s*CHUNK_THREADS + tid], the
// first cnt entries of a compacted list), bit s of the result set when that
// element is live and admitted (and, with a threshold T, its key >= T)
template <bool SCORE = true>
__device__ __forceinline__ uint32_t score_elems(const RankQ& Q, const NormState& N, int64_t c, int32_t* flagc,
                                                uint64_t* a, uint64_t* z, uint64_t T = 0,
                                                const PruneP* P = nullptr, const CardTab* tab = nullptr,
                                                const int16_t* idx = nullptr, int32_t cnt = 0) {
  const FilterQ* F = Q.filt;
  uint32_t vm = 0;
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++) {
    const int i = s * CHUNK_THREADS + (int)threadIdx.x;
    a[s] = 0;
    if (z) z[s] = 0;
    int64_t e;
    if (idx) {
      if (i >= cnt) continue;
      e = c * CHUNK + idx[i];
    } else {
      e = c * CHUNK + i;
      if (e >= Q.n || (Q.removed && ldg(Q.removed + e))) continue;
    }
    const Rec q = load_rec(Q.feat, e);
    uint64_t khi = 0;
    uint32_t klo = 0;
    if (F) {
      key_at(Q, e, khi, klo);
      if (!admit(*F, decode_rec(q), khi, klo, flagc)) continue;
    }
    if (!SCORE) continue;
    // below the query's threshold by an exact upper bound: no cardinal needed
    if (T && P && P->ok) {
      bool valid;
      const int64_t ub = score_bound(q, N, Q, *P, &valid, tab);
      if (valid && ((uint64_t)ub ^ 0x8000000000000000ull) < T) continue;
    }
    if (!F && Q.want_authority && !Q.host_rec && !Q.ecnt) key_at(Q, e, khi, klo);
    const Feat t = decode_rec(q);
    const int32_t hc = !Q.want_authority ? 0
                       : Q.ecnt ? ldg(Q.ecnt + e)
                                : host_count(Q, Q.host_rec ? q.w[3] >> 34 : key_host36(khi, klo));
    a[s] = (uint64_t)cardinal(t, N, Q, hc, tab) ^ 0x8000000000000000ull;
    if (a[s] < T) {
      a[s] = 0;
      continue;
    }
    if (z) z[s] = ((uint64_t)((uint32_t)q.w[3] ^ 0x80000000u) << 32) | (uint64_t)(~((uint32_t)e | Q.idx_tag));
    vm |= 1u << s;
  }
  return vm;
}

// With the query's threshold T known (and no filters): the chunk's live elements
// whose exact upper bound (score_bound, from words 2-3 of the record) reaches T,
// compacted into idx (chunk-local indices); returns their count.  cardinal
// then runs on dense waves of survivors instead of on every wave for a few lanes.
__device__ __forceinline__ int32_t prune_chunk(const RankQ& Q, const NormState& N, int64_t c, uint64_t T,
                                               const PruneP& P, const CardTab* tab, int16_t* idx, int32_t* sScan) {
  uint32_t keep = 0;
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++) {
    const int i = s * CHUNK_THREADS + (int)threadIdx.x;  // coalesced; the order of idx does not matter
    const int64_t e = c * CHUNK + i;
    if (e >= Q.n || (Q.removed && ldg(Q.removed + e))) continue;
    const ulonglong2 w23 = ldg(reinterpret_cast<const ulonglong2*>(Q.feat + e * FEAT_WORDS) + 1);
    Rec q;
    q.w[0] = q.w[1] = 0;
    q.w[2] = w23.x;
    q.w[3] = w23.y;
    bool valid;
    const int64_t ub = score_bound(q, N, Q, P, &valid, tab);
    if (!(valid && ((uint64_t)ub ^ 0x8000000000000000ull) < T)) keep |= 1u << s;
  }
  int32_t tot;
  int32_t o = block_excl_sum<CHUNK_THREADS>(__popc(keep), sScan, &tot);
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++)
    if ((keep >> s) & 1u) idx[o++] = (int16_t)(s * CHUNK_THREADS + (int)threadIdx.x);
  __syncthreads();
  return tot;
}


// MSB-first radix select over the live keys: the largest T with at least kq live keys >= T.
// With cap > 0 the select stops at the first digit whose bin takes the count of
// keys >= the bin's lowest key to at most cap: T is then that lowest key, a
// threshold with kq..cap keys above it (k_score sorts whatever T selects, so any
// such T is exact for it; fewer passes, each 3 barriers and a histogram).
__device__ __forceinline__ uint64_t score_threshold(const uint64_t* a, uint32_t vm, int32_t kq, int32_t* sHist,
                                                    int32_t* sSel, uint64_t* sRed, int32_t cap = 0) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint64_t mx = 0, mn = ~0ull;
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++)
    if ((vm >> s) & 1u) { mx = a[s] > mx ? a[s] : mx; mn = a[s] < mn ? a[s] : mn; }
  mx = wave_max_u64(mx);
  mn = wave_min_u64(mn);
  if (lane == 0) { sRed[wv] = mx; sRed[4 + wv] = mn; }
  __syncthreads();
  uint64_t gmx = sRed[0], gmn = sRed[4];
  for (int w = 1; w < 4; w++) { gmx = sRed[w] > gmx ? sRed[w] : gmx; gmn = sRed[4 + w] < gmn ? sRed[4 + w] : gmn; }
  const uint64_t diff = gmx ^ gmn;
  if (diff == 0) return gmx;
  int hi = 64 - __clzll((long long)diff);  // keys differ only in bits [0, hi)
  uint64_t prefix = hi == 64 ? 0 : (gmx >> hi) << hi;
  int32_t rem = kq;
  while (hi > 0) {
    const int lo = hi > 8 ? hi - 8 : 0;
    const uint32_t wmask = (1u << (hi - lo)) - 1u;
    sHist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < CHUNK_IPT; s++)
      if (((vm >> s) & 1u) && (hi == 64 || (a[s] >> hi) == (prefix >> hi)))
        atomicAdd(&sHist[(uint32_t)(a[s] >> lo) & wmask], 1);
    __syncthreads();
    if (tid < 64) radix_pick(sHist, rem, sSel);
    __syncthreads();
    prefix |= (uint64_t)sSel[0] << lo;
    if (cap > 0 && kq - sSel[1] + sSel[2] <= cap) return prefix;  // keys above the bin + the whole bin
    rem = sSel[1];
    hi = lo;
  }
  return prefix;
}


// Chunks run in `order` (every query's first chunks before anybody's later ones),
// so a big query's later chunks find its threshold (Tq, see PruneP) established.
__global__ __launch_bounds__(CHUNK_THREADS) void k_score(const RankQ* __restrict__ qs,
                                                        const int32_t* __restrict__ chunk_q,
                                                        const int32_t* __restrict__ order,
                                                        const NormState* __restrict__ norm, Cand* __restrict__ cand,
                                                        int32_t* __restrict__ cand_cnt, int32_t kc,
                                                        int32_t* __restrict__ redo, int32_t* __restrict__ nredo,
                                                        unsigned long long* __restrict__ Tq,
                                                        const QTab* __restrict__ qtab) {
  __shared__ uint64_t s1[SCORE_SMALL];
  __shared__ uint64_t s2[SCORE_SMALL];
  __shared__ int32_t sScan[4];
  __shared__ int32_t sHist[256];
  __shared__ int32_t sSel[3];
  __shared__ uint64_t sRed[8];
  __shared__ int32_t sFlag[32];
  __shared__ PruneP sP;
  __shared__ uint64_t sT;
  __shared__ CardTab sCard;
  __shared__ int16_t sIdx[CHUNK];  // prune_chunk's survivors (chunk-local)
  const int tid = threadIdx.x;
#ifdef YRWI_PHASE_CLOCK
  if (threadIdx.x == 0 && blockIdx.x < PH_MAXB) g_ts[blockIdx.x * 8] = wall_clock64();
#endif
  const int2 ob = reinterpret_cast<const int2*>(order)[blockIdx.x];  // (chunk, its query): one load
  const int64_t b = ob.x;
  const int qi = ob.y;
  const RankQ& Q = qs[qi];
  const NormState& N = norm[qi];  // per-query constants: scalar loads
  const int64_t c = b - Q.chunk_base;
  const int32_t kq = Q.k < kc ? Q.k : kc;
  // the one-byte fields' term tables pay off only for a chunk with many postings
  // (2304 entries per workgroup); a short chunk computes its few cardinals directly
  const int64_t nel = Q.n - c * CHUNK < CHUNK ? Q.n - c * CHUNK : CHUNK;
  const CardTab* tab = kq <= SCORE_SMALL && nel > YRWI_CARD_TAB_MIN ? &sCard : nullptr;  // workgroup-uniform
  if (tid == 0) {
    sT = __hip_atomic_load(Tq + qi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sP = qtab[qi].P;
  }
  if (tid < 32) sFlag[tid] = 0;
  if (tab) copy_card_tab(&sCard, &qtab[qi].T);
  __syncthreads();
  const FilterQ* F = Q.filt;
  int32_t* flagc = (F && F->flagcount) ? sFlag : nullptr;
  // strided element map (neighbouring lanes read neighbouring rows); the
  // candidate key carries the container index.  The hashCode (tie-break) is only
  // computed for the selected prefix.
  uint64_t a[CHUNK_IPT];
  if (kq > SCORE_SMALL) {  // large k (doubledom stacks): only the flag counts here
    if (flagc) {
      (void)score_elems<false>(Q, N, c, flagc, a, nullptr);
      __syncthreads();
      if (tid < 32 && sFlag[tid]) atomicAdd(&F->flagcount[tid], sFlag[tid]);
    }
    if (tid == 0) redo[atomicAdd(nredo, 1)] = (int32_t)b;
    return;
  }
  const PruneP P = sP;
  const uint64_t T0 = sT;
  PHASE(5)
  const bool comp = T0 && P.ok && !F;
  const int32_t nc = comp ? prune_chunk(Q, N, c, T0, P, tab, sIdx, sScan) : 0;
  const uint32_t vm = comp ? score_elems(Q, N, c, flagc, a, nullptr, T0, nullptr, tab, sIdx, nc)
                           : score_elems(Q, N, c, flagc, a, nullptr, T0, &P, tab);
  int32_t nv;
  int32_t voff = block_excl_sum<CHUNK_THREADS>(__popc(vm), sScan, &nv);  // (its barriers also order the sFlag atomics)
  PHASE(0)
  if (flagc && tid < 32 && sFlag[tid]) atomicAdd(&F->flagcount[tid], sFlag[tid]);
  if (kq <= 0 || nv == 0) {
    if (tid == 0) cand_cnt[b] = 0;
    return;
  }
  if (nv <= kq && Q.nchunks > 1) {
    // nothing to cut: every live candidate goes to k_topq as it is (k_topq sorts
    // and dedupes the union of a query's lists; only a single-chunk query's list
    // is final and must leave here sorted and deduped)
    Cand* out = cand + b * (int64_t)kc;
#pragma unroll
    for (int s = 0; s < CHUNK_IPT; s++)
      if ((vm >> s) & 1u) {
        const int i = s * CHUNK_THREADS + tid;
        const int64_t e = c * CHUNK + (comp ? sIdx[i] : i);
        const uint32_t h = (uint32_t)ldg(Q.feat + e * FEAT_WORDS + 3);  // ByteArray.hashCode (ByteArray.java:80-84)
        out[voff].k1 = a[s];
        out[voff].k2 = ((uint64_t)(h ^ 0x80000000u) << 32) | (uint64_t)(~((uint32_t)e | Q.idx_tag));
        voff++;
      }
    if (tid == 0) cand_cnt[b] = nv;
    return;
  }
  const uint64_t T = nv > kq ? score_threshold(a, vm, kq, sHist, sSel, sRed, SCORE_CAP) : 0;
  PHASE(1)
  int32_t mine = 0;
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++) mine += (((vm >> s) & 1u) && a[s] >= T) ? 1 : 0;
  int32_t nsel;
  int32_t off = block_excl_sum<CHUNK_THREADS>(mine, sScan, &nsel);
  if (nsel > SCORE_SMALL) {  // long run of tied scores at the cut
    if (tid == 0) redo[atomicAdd(nredo, 1)] = (int32_t)b;
    return;
  }
#pragma unroll
  for (int s = 0; s < CHUNK_IPT; s++)
    if (((vm >> s) & 1u) && a[s] >= T) {
      const int i = s * CHUNK_THREADS + tid;
      const int64_t e = c * CHUNK + (comp ? sIdx[i] : i);
      const uint32_t h = (uint32_t)ldg(Q.feat + e * FEAT_WORDS + 3);  // ByteArray.hashCode (ByteArray.java:80-84)
      s1[off] = a[s];
      s2[off] = ((uint64_t)((uint32_t)h ^ 0x80000000u) << 32) | (uint64_t)(~((uint32_t)e | Q.idx_tag));
      off++;
    }
  const int NP = pow2_at_least(nsel);
  for (int i = nsel + tid; i < NP; i += CHUNK_THREADS) { s1[i] = 0; s2[i] = 0; }
  __syncthreads();
  PHASE(2)
  bitonic_desc<CHUNK_THREADS>(s1, s2, NP);
  PHASE(3)
  int32_t distinct;
  Cand* out = cand + b * (int64_t)kc;
  const int32_t n = dedupe_take<CHUNK_THREADS>(s1, s2, NP, kq, out, sScan, &distinct, Tq + qi);
  PHASE(4)
  if (distinct < kq && nsel < nv) {  // the TreeSet dedupe consumed part of the prefix
    if (tid == 0) redo[atomicAdd(nredo, 1)] = (int32_t)b;
    return;
  }
  if (tid == 0) cand_cnt[b] = n;
}

// The chunks k_score could not finish, whole chunk in LDS (grid-stride over the redo list).
__global__ __launch_bounds__(CHUNK_THREADS) void k_score_full(const RankQ* __restrict__ qs,
                                                             const int32_t* __restrict__ chunk_q,
                                                             const NormState* __restrict__ norm,
                                                             Cand* __restrict__ cand, int32_t* __restrict__ cand_cnt,
                                                             int32_t kc, const int32_t* __restrict__ redo,
                                                             const int32_t* __restrict__ nredo) {
  __shared__ uint64_t s1[CHUNK];
  __shared__ uint64_t s2[CHUNK];
  __shared__ int32_t sScan[4];
  __shared__ int32_t sHist[256];
  __shared__ int32_t sSel[3];
  __shared__ uint64_t sRed[8];
  __shared__ CardTab sCard;
  const int tid = threadIdx.x;
  const int32_t nr = *nredo;
  for (int32_t ri = blockIdx.x; ri < nr; ri += gridDim.x) {
    const int64_t b = redo[ri];
    const int qi = chunk_q[b];
    const RankQ& Q = qs[qi];
    const NormState& N = norm[qi];
    __syncthreads();  // LDS of the previous chunk
    build_card_tab(&sCard, N, Q);
    __syncthreads();
    const int64_t c = b - Q.chunk_base;
    uint64_t a[CHUNK_IPT], z[CHUNK_IPT];
    const uint32_t vm = score_elems(Q, N, c, nullptr, a, z, 0, nullptr, &sCard);  // flags were counted by k_score
    const int32_t kq = Q.k < kc ? Q.k : kc;
    int32_t nv;
    (void)block_excl_sum<CHUNK_THREADS>(__popc(vm), sScan, &nv);
    const uint64_t T = nv > kq ? score_threshold(a, vm, kq, sHist, sSel, sRed) : 0;
    int32_t mine = 0;
#pragma unroll
    for (int s = 0; s < CHUNK_IPT; s++) mine += (((vm >> s) & 1u) && a[s] >= T) ? 1 : 0;
    int32_t nsel;
    int32_t off = block_excl_sum<CHUNK_THREADS>(mine, sScan, &nsel);
#pragma unroll
    for (int s = 0; s < CHUNK_IPT; s++)
      if (((vm >> s) & 1u) && a[s] >= T) { s1[off] = a[s]; s2[off] = z[s]; off++; }
    const int P = pow2_at_least(nsel);
    for (int i = nsel + tid; i < P; i += CHUNK_THREADS) { s1[i] = 0; s2[i] = 0; }
    __syncthreads();
    bitonic_desc<CHUNK_THREADS>(s1, s2, P);
    Cand* out = cand + b * (int64_t)kc;
    int32_t distinct;
    int32_t n = dedupe_take<CHUNK_THREADS>(s1, s2, P, kq, out, sScan, &distinct);
    if (distinct < kq && nsel < nv) {
      // the TreeSet dedupe consumed part of the prefix: sort the whole chunk
      __syncthreads();
#pragma unroll
      for (int s = 0; s < CHUNK_IPT; s++) { s1[tid * CHUNK_IPT + s] = a[s]; s2[tid * CHUNK_IPT + s] = z[s]; }
      __syncthreads();
      bitonic_desc<CHUNK_THREADS>(s1, s2, CHUNK);
      n = dedupe_take<CHUNK_THREADS>(s1, s2, CHUNK, kq, out, sScan, nullptr);
    }
    if (tid == 0) cand_cnt[b] = n;
  }
}

// Top-k of a group of candidate lists (gn[g] <= 64 lists from list gbase[g];
// each list <= its stride kc entries, in any order and not necessarily deduped --
// the union is selected, sorted and deduped here; k = gk[g]; the host sizes
// groups to <= CAP candidates), in rounds.  The group's candidates are staged in
// LDS; a round takes the r = k - emitted largest remaining candidates by the full
// 128-bit key (k1, k2) -- exact, keys are unique -- found by MSB-first radix
// select (k1 digits over the bits where the candidates differ, then k2 digits
// only if the cut falls inside a run of equal k1), moves them to the front,
// sorts them and applies the TreeSet dedupe against the predecessor (the previous
// round's last key at the boundary).  A further round (after re-staging) is
// needed only when the dedupe dropped candidates.
constexpr int TOPQ_THREADS = 256;

// radix select of the r-th largest 64-bit key among the members of the staged
// candidates; F(f, key&) -> member?
template <class F>
__device__ uint64_t topq_select(F key_at, int32_t total, int32_t r, uint64_t mx, uint64_t mn, int32_t nmem,
                                int32_t* grp, int32_t* rank, int32_t* sHist, int32_t* sSel) {
  const uint64_t diff = mx ^ mn;
  if (diff == 0) { *grp = nmem; *rank = r; return mx; }
  int hi = 64 - __clzll((long long)diff);
  uint64_t prefix = hi == 64 ? 0 : (mx >> hi) << hi;
  int32_t rem = r, g = nmem;
  while (hi > 0) {
    const int lo = hi > 8 ? hi - 8 : 0;
    const uint32_t wmask = (1u << (hi - lo)) - 1u;
    sHist[threadIdx.x] = 0;
    __syncthreads();
    for (int f = threadIdx.x; f < total; f += TOPQ_THREADS) {
      uint64_t key;
      if (key_at(f, key) && (hi == 64 || (key >> hi) == (prefix >> hi)))
        atomicAdd(&sHist[(uint32_t)(key >> lo) & wmask], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) radix_pick(sHist, rem, sSel);
    __syncthreads();
    prefix |= (uint64_t)sSel[0] << lo;
    rem = sSel[1];
    g = sSel[2];
    hi = lo;
    __syncthreads();
  }
  *grp = g;
  *rank = rem;
  return prefix;
}

__device__ __forceinline__ void block_minmax_u64(uint64_t& mx, uint64_t& mn, uint64_t* sRed) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  mx = wave_max_u64(mx);
  mn = wave_min_u64(mn);
  if (lane == 0) { sRed[wv] = mx; sRed[4 + wv] = mn; }
  __syncthreads();
  mx = sRed[0];
  mn = sRed[4];
  for (int w = 1; w < TOPQ_THREADS / 64; w++) { mx = sRed[w] > mx ? sRed[w] : mx; mn = sRed[4 + w] < mn ? sRed[4 + w] : mn; }
  __syncthreads();
}

template <int CAP>
__global__ __launch_bounds__(TOPQ_THREADS) void k_topq(const int64_t* __restrict__ gbase, const int32_t* __restrict__ gn,
                                                      const int32_t* __restrict__ gk, const Cand* __restrict__ cand,
                                                      const int32_t* __restrict__ ccnt, int32_t kc, int32_t keff,
                                                      Cand* __restrict__ out, int32_t* __restrict__ out_cnt) {
  constexpr int EPT = CAP / TOPQ_THREADS;
  extern __shared__ uint64_t smem[];
  uint64_t* c1 = smem;
  uint64_t* c2 = smem + CAP;
  __shared__ int32_t sHist[256];
  __shared__ int32_t sSel[3];
  __shared__ int32_t sScan[4];
  __shared__ int32_t sOff[65];
  __shared__ uint64_t sRed[8];
  const int tid = threadIdx.x;
  const int64_t g = blockIdx.x;
  const int32_t k = min(gk[g], keff);
  const int32_t nl = gn[g];
  const Cand* lists = cand + gbase[g] * kc;
  if (tid < 64) {
    const int32_t c = tid < nl ? ccnt[gbase[g] + tid] : 0;
    sOff[tid + 1] = wave_incl_sum(c);
    if (tid == 0) sOff[0] = 0;
  }
  __syncthreads();
  const int32_t total = sOff[nl];
  auto stage = [&]() {  // flatten the group's lists into c1/c2[0, total)
    for (int f = tid; f < total; f += TOPQ_THREADS) {
      int lo = 0, hi = nl - 1;  // largest l with sOff[l] <= f
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sOff[mid] <= f) lo = mid; else hi = mid - 1;
      }
      const Cand c = lists[(int64_t)lo * kc + (f - sOff[lo])];
      c1[f] = c.k1;
      c2[f] = c.k2;
    }
    __syncthreads();
  };
  stage();
  Cand* dst = out + g * keff;
  bool first = true;
  uint64_t U1 = 0, U2 = 0;  // exclusive upper bound: the previous round's smallest key
  int32_t emitted = 0;
  while (emitted < k) {
    auto inC = [&](uint64_t a, uint64_t z) { return first || a < U1 || (a == U1 && z < U2); };
    int32_t n = 0;
    uint64_t mx = 0, mn = ~0ull;
    for (int f = tid; f < total; f += TOPQ_THREADS)
      if (inC(c1[f], c2[f])) { n++; mx = c1[f] > mx ? c1[f] : mx; mn = c1[f] < mn ? c1[f] : mn; }
    int32_t nmem;
    (void)block_excl_sum<TOPQ_THREADS>(n, sScan, &nmem);
    if (nmem == 0) break;
    block_minmax_u64(mx, mn, sRed);
    const int32_t r = min(k - emitted, nmem);
    int32_t grp, rank;
    const uint64_t T1 = topq_select([&](int f, uint64_t& key) {
      if (!inC(c1[f], c2[f])) return false;
      key = c1[f];
      return true;
    }, total, r, mx, mn, nmem, &grp, &rank, sHist, sSel);
    uint64_t T2 = 0;
    if (rank < grp) {  // the cut falls inside the run k1 == T1: select on k2 there
      uint64_t zx = 0, zn = ~0ull;
      for (int f = tid; f < total; f += TOPQ_THREADS)
        if (c1[f] == T1 && inC(c1[f], c2[f])) { zx = c2[f] > zx ? c2[f] : zx; zn = c2[f] < zn ? c2[f] : zn; }
      block_minmax_u64(zx, zn, sRed);
      int32_t g2, r2;
      T2 = topq_select([&](int f, uint64_t& key) {
        if (c1[f] != T1 || !inC(c1[f], c2[f])) return false;
        key = c2[f];
        return true;
      }, total, rank, zx, zn, grp, &g2, &r2, sHist, sSel);
    }
    // move the r selected keys (exactly r: keys are unique) to the front, sort, dedupe
    uint64_t v1[EPT], v2[EPT];
    uint32_t selb = 0;
    int32_t mine = 0;
#pragma unroll
    for (int j = 0; j < EPT; j++) {
      const int f = j * TOPQ_THREADS + tid;
      v1[j] = 0;
      v2[j] = 0;
      if (f < total) {
        v1[j] = c1[f];
        v2[j] = c2[f];
        if (inC(v1[j], v2[j]) && (v1[j] > T1 || (v1[j] == T1 && v2[j] >= T2))) { selb |= 1u << j; mine++; }
      }
    }
    int32_t nsel;
    int32_t off = block_excl_sum<TOPQ_THREADS>(mine, sScan, &nsel);  // (its barriers order the reads above)
#pragma unroll
    for (int j = 0; j < EPT; j++)
      if (selb & (1u << j)) { c1[off] = v1[j]; c2[off] = v2[j]; off++; }
    const int P = pow2_at_least(nsel);
    for (int i = nsel + tid; i < P; i += TOPQ_THREADS) { c1[i] = 0; c2[i] = 0; }
    __syncthreads();
    bitonic_desc<TOPQ_THREADS>(c1, c2, P);
    const int ipt = (nsel + TOPQ_THREADS - 1) / TOPQ_THREADS;
    const int i0 = tid * ipt;
    int32_t keep = 0;
    uint32_t bits = 0;
    for (int t = 0; t < ipt; t++) {
      const int i = i0 + t;
      if (i >= nsel) break;
      const uint64_t p1 = i > 0 ? c1[i - 1] : U1, p2 = i > 0 ? c2[i - 1] : U2;
      const bool dup = (i > 0 || !first) && c1[i] == p1 && (c2[i] >> 32) == (p2 >> 32);
      if (!dup) { bits |= 1u << t; keep++; }
    }
    int32_t kept;
    off = block_excl_sum<TOPQ_THREADS>(keep, sScan, &kept);
    for (int t = 0; t < ipt; t++) {
      if (bits & (1u << t)) {
        if (emitted + off < k) { dst[emitted + off].k1 = c1[i0 + t]; dst[emitted + off].k2 = c2[i0 + t]; }
        off++;
      }
    }
    emitted = min(k, emitted + kept);
    U1 = c1[nsel - 1];
    U2 = c2[nsel - 1];
    first = false;
    __syncthreads();
    if (emitted < k) stage();  // the front of the image was overwritten
  }
  if (tid == 0) out_cnt[g] = emitted;
}

// Emit final candidates as yrwi_hit records.  mode EMIT_OUT: queries without
// doubledom, their first kout hits to `hits`; EMIT_STACK: every query's stack
// (k hits, the doubledom bound), input of the shard merge; EMIT_STACK_DD: only
// the doubledom queries' stacks (k_pull orders them).
enum : int { EMIT_OUT = 0, EMIT_STACK = 1, EMIT_STACK_DD = 2 };

__global__ void k_emit(const RankQ* __restrict__ qs, int nq, const Cand* const* __restrict__ fin,
                       const int32_t* const* __restrict__ fin_cnt, int32_t kmax, yrwi_hit* __restrict__ hits,
                       int32_t* __restrict__ nout, int mode) {
  const int qi = blockIdx.x;
  const RankQ& Q = qs[qi];
  if ((mode == EMIT_OUT && Q.doubledom) || (mode == EMIT_STACK_DD && !Q.doubledom)) return;
  const int32_t n = min(*fin_cnt[qi], min(mode == EMIT_OUT ? Q.kout : Q.k, kmax));
  const Cand* f = fin[qi];
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const Cand cd = f[i];
    const uint32_t idx = ~(uint32_t)cd.k2 & 0x0FFFFFFFu;
    uint64_t khi;
    uint32_t klo;
    key_at(Q, idx, khi, klo);
    yrwi_hit h;
    key_chars(khi, klo, h.urlhash);
    h.tiebreak = (int32_t)((uint32_t)(cd.k2 >> 32) ^ 0x80000000u);
    h.score = (int64_t)(cd.k1 ^ 0x8000000000000000ull);
    hits[(int64_t)qi * kmax + i] = h;
  }
  if (threadIdx.x == 0) nout[qi] = n;
}

// ------------------------------------------------ cross-shard merge (sharded)
// Gathered per-shard stacks allh[s][q][0, alln[s][q]) (each in rwiStack order)
// are merged as one TreeSet fed in url-hash (= shard) order: order (score desc,
// hashCode desc, shard asc); an entry whose (score, hashCode) already occurs in
// a lower shard is rejected.  k_gmerge_rank places every entry at its merged
// position (its index + the entries of the other shards ahead of it);
// k_gmerge_out compacts the survivors into the query's merged stack.
__device__ __forceinline__ bool hit_before(const yrwi_hit& x, int64_t score, int32_t tb, bool ties_first) {
  return x.score > score || (x.score == score && (x.tiebreak > tb || (ties_first && x.tiebreak == tb)));
}

__global__ void k_gmerge_rank(const yrwi_hit* __restrict__ allh, const int32_t* __restrict__ alln, int W, int nq,
                              int32_t kint, uint32_t* __restrict__ slot, uint8_t* __restrict__ dup) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)W * kint;
  if (t >= per * nq) return;
  const int q = (int)(t / per);
  const int s = (int)((t % per) / kint);
  const int32_t i = (int32_t)(t % kint);
  if (i >= alln[(int64_t)s * nq + q]) return;
  const yrwi_hit me = allh[((int64_t)s * nq + q) * kint + i];
  int64_t pos = i;
  uint8_t d = 0;
  for (int s2 = 0; s2 < W; s2++) {
    if (s2 == s) continue;
    const yrwi_hit* L = allh + ((int64_t)s2 * nq + q) * kint;
    const int32_t n2 = alln[(int64_t)s2 * nq + q];
    const bool ties_first = s2 < s;  // a lower shard's equal key precedes
    int32_t lo = 0, hi = n2;         // first element not before me
    while (lo < hi) {
      const int32_t m = (lo + hi) >> 1;
      if (hit_before(L[m], me.score, me.tiebreak, ties_first)) lo = m + 1; else hi = m;
    }
    pos += lo;
    if (ties_first && lo > 0 && L[lo - 1].score == me.score && L[lo - 1].tiebreak == me.tiebreak) d = 1;
  }
  slot[(int64_t)q * per + pos] = (uint32_t)(s * kint + i);
  dup[(int64_t)q * per + pos] = d;
}

__global__ __launch_bounds__(256) void k_gmerge_out(const RankQ* __restrict__ qs, const yrwi_hit* __restrict__ allh,
                                                    const int32_t* __restrict__ alln, int W, int nq, int32_t kint,
                                                    const uint32_t* __restrict__ slot, const uint8_t* __restrict__ dup,
                                                    yrwi_hit* __restrict__ stack, int32_t* __restrict__ scnt) {
  __shared__ int32_t sScan[4];
  const int q = blockIdx.x;
  const RankQ& Q = qs[q];
  const int64_t per = (int64_t)W * kint;
  int32_t T = 0;
  for (int s = 0; s < W; s++) T += alln[(int64_t)s * nq + q];
  const int32_t lim = min(Q.k, kint);
  int32_t base = 0;
  for (int32_t c0 = 0; c0 < T && base < lim; c0 += 256) {
    const int32_t p = c0 + (int32_t)threadIdx.x;
    const int keep = (p < T && !dup[(int64_t)q * per + p]) ? 1 : 0;
    int32_t tot;
    const int32_t off = block_excl_sum256(keep, sScan, &tot);
    if (keep && base + off < lim) {
      const uint32_t sl = slot[(int64_t)q * per + p];
      const int s = (int)(sl / (uint32_t)kint), i = (int)(sl % (uint32_t)kint);
      stack[(int64_t)q * kint + base + off] = allh[((int64_t)s * nq + q) * kint + i];
    }
    base += tot;
  }
  if (threadIdx.x == 0) scnt[q] = min(base, lim);
}

// ------------------------------------------------ result pulling
// pullOneRWI(skipDoubleDom = true) repeated kout times over the settled stack
// (SearchEvent.java:1297-1394).  Each round polls up to 10 stack entries; the
// first one of a host without a doubleDomCache entry is returned (the host gets
// an entry), the others are queued on their host.  A round that returns nothing
// takes the best queued entry -- the earliest queued one, since the stack is in
// rank order (equal weights: the earliest) -- and a host whose queue
// runs empty leaves the cache.  The queues together are one FIFO in stack order.
// One workgroup per query: hosts are interned in an LDS hash table in parallel,
// then lane 0 replays the pull sequence on small LDS arrays.  Queries without
// doubledom just copy the first kout entries (only_dd = 0).
constexpr int DD_SLOTS = 8192;  // > 2 * YRWI_MAX_K

__device__ __forceinline__ uint64_t hit_host36(const yrwi_hit& h) {
  uint64_t x = 0;
#pragma unroll
  for (int j = 6; j < 12; j++) x = (x << 6) | (uint64_t)(ahpla(h.urlhash[j]) & 63);
  return x;
}

__global__ __launch_bounds__(64) void k_pull(const RankQ* __restrict__ qs, const yrwi_hit* __restrict__ stack,
                                             const int32_t* __restrict__ scnt, int32_t kint, int only_dd,
                                             int32_t kmax, yrwi_hit* __restrict__ hits, int32_t* __restrict__ nout) {
  __shared__ unsigned long long sKey[DD_SLOTS];
  __shared__ uint16_t sCnt[DD_SLOTS];     // queued entries of the host
  __shared__ uint8_t sSeen[DD_SLOTS];     // host has a doubleDomCache entry
  __shared__ uint16_t sHost[YRWI_MAX_K];  // stack position -> host slot
  __shared__ uint16_t sFifo[YRWI_MAX_K];
  __shared__ uint16_t sOut[YRWI_MAX_K];
  __shared__ int32_t sN;
  const int qi = blockIdx.x;
  const RankQ& Q = qs[qi];
  if (only_dd && !Q.doubledom) return;
  const yrwi_hit* st = stack + (int64_t)qi * kint;
  const int32_t n = min(scnt[qi], min((int32_t)YRWI_MAX_K, kint));
  const int32_t want = min(Q.kout, kmax);
  if (!Q.doubledom) {
    const int32_t m = min(n, want);
    for (int o = threadIdx.x; o < m; o += 64) hits[(int64_t)qi * kmax + o] = st[o];
    if (threadIdx.x == 0) nout[qi] = m;
    return;
  }
  for (int i = threadIdx.x; i < DD_SLOTS; i += 64) { sKey[i] = 0; sCnt[i] = 0; sSeen[i] = 0; }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 64) {
    const uint64_t key = hit_host36(st[i]) + 1;
    uint32_t slot = (uint32_t)mix64(key) & (DD_SLOTS - 1);
    while (true) {
      const unsigned long long prev = atomicCAS(&sKey[slot], 0ull, (unsigned long long)key);
      if (prev == 0ull || prev == key) break;
      slot = (slot + 1) & (DD_SLOTS - 1);
    }
    sHost[i] = (uint16_t)slot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t out = 0, i = 0, qh = 0, qt = 0;
    while (out < want) {
      int32_t got = -1;
      for (int c = 0; i < n && c < 10; c++) {
        const int32_t pos = i++;
        const int h = sHost[pos];
        if (!sSeen[h]) { sSeen[h] = 1; got = pos; break; }
        sCnt[h]++;
        sFifo[qt++] = (uint16_t)pos;
      }
      if (got >= 0) { sOut[out++] = (uint16_t)got; continue; }
      if (qh == qt) break;
      const int32_t pos = sFifo[qh++];
      const int h = sHost[pos];
      if (--sCnt[h] == 0) sSeen[h] = 0;
      sOut[out++] = (uint16_t)pos;
    }
    sN = out;
  }
  __syncthreads();
  const int32_t m = sN;
  for (int o = threadIdx.x; o < m; o += 64) hits[(int64_t)qi * kmax + o] = st[sOut[o]];
  if (threadIdx.x == 0) nout[qi] = m;
}


// all scores of a container (yrwi_normalize_score)
__global__ __launch_bounds__(256) void k_score_all(const RankQ* __restrict__ qs,
                                                   const int32_t* __restrict__ chunk_q,
                                                   const NormState* __restrict__ norm, int64_t* __restrict__ out) {
  const int64_t b = blockIdx.x;
  const int qi = chunk_q[b];
  const RankQ& Q = qs[qi];
  const NormState N = norm[qi];
  const int64_t c = b - Q.chunk_base;
  for (int s = threadIdx.x; s < CHUNK; s += blockDim.x) {
    const int64_t e = c * CHUNK + s;
    if (e >= Q.n) break;
    const Rec q = load_rec(Q.feat, e);
    const Feat t = decode_rec(q);
    const int32_t hc = !Q.want_authority ? 0 : Q.ecnt ? ldg(Q.ecnt + e) : host_count(Q, elem_host(Q, q.w[3], e));
    out[e] = cardinal(t, N, Q, hc);
  }
}

// ======================================================= host-count exchange
// Global host counts for ReferenceOrder.authority (:176-216) when the joined
// container is spread over url-hash shards: every (query, host, local count) is
// sent to the host's owner rank, summed there and the totals are sent back.
__device__ __forceinline__ uint32_t owner_of(uint64_t key, int world) {
  return (uint32_t)((mix64(key ^ 0x5BD1E995ull) >> 32) % (uint64_t)world);
}

// a host table's slot key as the exchange names hosts (host hash + 1): tables of
// dense host ids (host_key != nullptr) translate theirs
__device__ __forceinline__ uint64_t slot_host(uint64_t k, const uint64_t* __restrict__ host_key) {
  return (k && host_key) ? host_key[k - 1] + 1 : k;
}

__global__ void k_host_count(const uint64_t* __restrict__ hkeys, int64_t nslots, int world,
                             uint32_t* __restrict__ owner_cnt, const uint64_t* __restrict__ host_key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots) return;
  const uint64_t k = slot_host(hkeys[i], host_key);
  if (k) atomicAdd(&owner_cnt[owner_of(k, world)], 1u);
}

__global__ void k_host_pack(const uint64_t* __restrict__ hkeys, const uint32_t* __restrict__ hcnt,
                            const int64_t* __restrict__ slot_base, int nq, int64_t nslots, int world,
                            uint32_t* __restrict__ cursor, HostMsg* __restrict__ send,
                            uint64_t* __restrict__ send_slot, const uint64_t* __restrict__ host_key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots) return;
  const uint64_t k = slot_host(hkeys[i], host_key);
  if (!k) return;
  const int q = find_job(slot_base, nq, i);
  const uint32_t pos = atomicAdd(&cursor[owner_of(k, world)], 1u);
  send[pos] = HostMsg{k, (uint32_t)q, hcnt[i]};
  send_slot[pos] = (uint64_t)i;
}

__device__ __forceinline__ uint64_t owner_key(const HostMsg& m) { return ((uint64_t)m.q << 37) | m.key; }

__global__ void k_host_insert(const HostMsg* __restrict__ recv, int64_t n, uint64_t* __restrict__ okeys,
                              uint32_t* __restrict__ ocnt, uint64_t omask) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const HostMsg m = recv[i];
  const uint64_t ck = owner_key(m);
  uint64_t slot = mix64(ck) & omask;
  while (true) {
    unsigned long long prev = atomicCAS((unsigned long long*)&okeys[slot], 0ull, (unsigned long long)ck);
    if (prev == 0ull || prev == ck) {
      atomicAdd(&ocnt[slot], m.cnt);
      return;
    }
    slot = (slot + 1) & omask;
  }
}

__global__ void k_host_max(const uint64_t* __restrict__ okeys, const uint32_t* __restrict__ ocnt, int64_t ocap,
                           int32_t* __restrict__ gmax) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ocap) return;
  const uint64_t ck = okeys[i];
  if (ck) atomicMax(&gmax[ck >> 37], (int32_t)ocnt[i]);
}

__global__ void k_host_reply(const HostMsg* __restrict__ recv, int64_t n, const uint64_t* __restrict__ okeys,
                             const uint32_t* __restrict__ ocnt, uint64_t omask, uint32_t* __restrict__ reply) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t ck = owner_key(recv[i]);
  uint64_t slot = mix64(ck) & omask;
  while (okeys[slot] != ck) slot = (slot + 1) & omask;  // present: inserted above
  reply[i] = ocnt[slot];
}

__global__ void k_host_apply(const uint32_t* __restrict__ back, const uint64_t* __restrict__ send_slot, int64_t n,
                             uint32_t* __restrict__ hcnt_all) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) hcnt_all[send_slot[i]] = back[i];
}

__global__ void k_set_maxdom(ShardSum* __restrict__ ss, const int32_t* __restrict__ gmax, int nq) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < nq) ss[q].maxdom = gmax[q];
}

// ================================================================ launchers
static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline int rc(hipError_t e) { return e == hipSuccess ? 0 : YRWI_E_HIP; }

int launch_validate_rows(const uint8_t* rows, int64_t n, uint64_t* khi, uint8_t* klo, int32_t* err, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_validate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), rows, n, khi, klo, err);
  return rc(hipGetLastError());
}

int launch_features(const uint8_t* rows, int64_t n, uint64_t* feat, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_features, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), rows, n, feat);
  return rc(hipGetLastError());
}

int launch_feat_rows(const uint64_t* feat, const uint32_t* uid, const uint64_t* dkhi, const uint8_t* dklo, int64_t n,
                     int64_t now_ms, uint8_t* rows, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_feat_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), feat, uid, dkhi, dklo, n,
                     now_ms, rows);
  return rc(hipGetLastError());
}

int launch_join_step(const JoinQ* d_jobs, const int64_t* d_tile_base, int32_t njobs, int32_t nmerge,
                     int64_t merge_tiles, int64_t total_tiles, TileDesc* d_desc, ProbeDesc* d_pdesc,
                     uint2* d_pairs, uint32_t* d_pair_uid, int64_t* d_tile_src, int32_t* d_tile_cnt,
                     int64_t* d_tile_off, bool mark, bool long_tiles, const BandOrder& bo,
                     void* st, void* ev0,
                     void* evm, void* ev1, void* evc0, void* evc1, bool chain, int32_t* d_tile_lvl,
                     ProbeDesc* d_crange, const int2* d_cgrp, int64_t ngroups, BmFast* d_fast,
                     BmFast* d_fast_perm, int sum) {
  if (total_tiles <= 0) return 0;
  const int64_t probe_tiles = total_tiles - merge_tiles;
  // band orders (k_order_hist / k_order_scatter): all tiles for k_compact, probe tiles for k_probe
  int2* perm = bo.key && bo.tile_job && !mark ? bo.perm : nullptr;
  int2* pperm = bo.pkey && bo.tile_job && probe_tiles > 1 ? bo.pperm : nullptr;
  uint32_t* tkey = perm ? bo.key : nullptr;
  uint32_t* pkey = pperm ? bo.pkey : nullptr;
  int32_t* tjob = bo.tile_job;
  static int join_grid = 0;  // resident k_join workgroups on the whole device
  if (!join_grid) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&k_join), JOIN_THREADS,
                                                     0) != hipSuccess)
      return YRWI_E_HIP;
    join_grid = std::max(1, cus * std::max(1, per_cu));
  }
  if (merge_tiles > 0) {
    hipLaunchKernelGGL(k_partition, dim3((unsigned)((merge_tiles + 255) / 256)), dim3(256), 0, S(st), d_jobs,
                       d_tile_base, nmerge, merge_tiles, d_desc, d_tile_src, tkey, tjob);
    if (!mark) hipLaunchKernelGGL(k_scan_bounds, dim3((unsigned)nmerge), dim3(256), 0, S(st), d_jobs, d_tile_base, d_tile_src);
  }
  if (probe_tiles > 0)
    hipLaunchKernelGGL(k_probe_part, dim3((unsigned)((probe_tiles + 255) / 256)), dim3(256), 0, S(st), d_jobs,
                       d_tile_base, njobs, merge_tiles, probe_tiles, d_pdesc, tkey, tjob, pkey, bo.pshift,
                       mark ? nullptr : d_fast);
  if (perm || pperm) {
    OrderArgs oa{};
    int nb = 0;
    auto prob = [&](int i, const uint32_t* key, int64_t n, int shift, const int32_t* job, int2* out,
                    const BmFast* pay = nullptr, BmFast* pay_out = nullptr) {
      OrderProb& P = oa.p[i];
      P.pay = pay;
      P.pay_out = pay_out;
      P.key = key;
      P.n = n;
      P.nslices = (int32_t)std::min<int64_t>(64, (n + ORDER_SLICE_MIN - 1) / ORDER_SLICE_MIN);
      P.slice = (n + P.nslices - 1) / P.nslices;
      P.shift = shift;
      P.tile_job = job;
      P.perm = out;
      P.hist = bo.hist + (int64_t)nb * ORDER_BUCKETS;
      nb += P.nslices;
    };
    if (perm) prob(0, tkey, total_tiles, bo.shift, tjob, perm);
    if (pperm)
      prob(perm ? 1 : 0, pkey, probe_tiles, 0, tjob + merge_tiles, pperm, mark ? nullptr : d_fast,
           mark ? nullptr : d_fast_perm);
    hipLaunchKernelGGL(k_order_hist, dim3((unsigned)nb), dim3(ORDER_THREADS), 0, S(st), oa);
    hipLaunchKernelGGL(k_order_scatter, dim3((unsigned)nb), dim3(ORDER_THREADS), 0, S(st), oa);
  }
  if (ev0) hipEventRecord(reinterpret_cast<hipEvent_t>(ev0), S(st));
  if (merge_tiles > 0)
    hipLaunchKernelGGL(k_join, dim3((unsigned)std::min<int64_t>(merge_tiles, join_grid)), dim3(JOIN_THREADS), 0,
                       S(st), d_jobs, d_desc, merge_tiles, d_pairs, d_pair_uid, d_tile_src, d_tile_cnt, mark ? 1 : 0);
  if (evm) hipEventRecord(reinterpret_cast<hipEvent_t>(evm), S(st));
  if (probe_tiles > 0) {
    auto kp = long_tiles ? (mark ? k_probe<true, true> : k_probe<true, false>)
                         : (mark ? k_probe<false, true> : k_probe<false, false>);
    const BmFast* fast = mark || !d_fast ? nullptr : pperm ? d_fast_perm : d_fast;  // (k_probe's order)
    hipLaunchKernelGGL(kp, dim3((unsigned)probe_tiles), dim3(PROBE_TILE), 0, S(st), d_jobs, d_tile_base, d_pdesc,
                       merge_tiles, d_pairs, d_pair_uid, d_tile_src, d_tile_cnt, (const int2*)pperm, d_tile_lvl, fast);
  }
  if (ev1) hipEventRecord(reinterpret_cast<hipEvent_t>(ev1), S(st));
  if (!mark) {
    if (chain && ngroups > 0) {  // chain groups
      const int64_t nr = ngroups * CHAIN_MAXL;
      hipLaunchKernelGGL(k_chain_part, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, S(st), d_jobs,
                         d_tile_base, njobs, d_cgrp, ngroups, (const uint32_t*)d_pair_uid,
                         (const int64_t*)d_tile_src, (const int32_t*)d_tile_cnt, d_crange);
      // chained steps: evc0 / evc1 bracket k_chain alone (the population rocprofv3 averages)
      if (evc0) hipEventRecord(reinterpret_cast<hipEvent_t>(evc0), S(st));
      hipLaunchKernelGGL(k_chain, dim3((unsigned)ngroups), dim3(256), 0, S(st), d_jobs, d_tile_base, njobs, d_cgrp,
                         d_pairs, d_pair_uid, d_tile_src, d_tile_cnt, d_tile_lvl, (const ProbeDesc*)d_crange);
      if (evc1) hipEventRecord(reinterpret_cast<hipEvent_t>(evc1), S(st));
    }
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)njobs), dim3(256), 0, S(st), d_jobs, d_tile_base, d_tile_cnt,
                       d_tile_off, (const int32_t*)(chain ? d_tile_lvl : nullptr));
    if (!chain) {  // chained steps compact once the fold's dispatch modes are known (launch_compact)
      if (evc0) hipEventRecord(reinterpret_cast<hipEvent_t>(evc0), S(st));
      if (int r = launch_compact(d_jobs, d_tile_base, njobs, total_tiles, d_pairs, d_pair_uid, d_tile_src, d_tile_cnt,
                                 d_tile_off, bo, false, st, sum))
        return r;
      if (evc1) hipEventRecord(reinterpret_cast<hipEvent_t>(evc1), S(st));
    }
  }
  return rc(hipGetLastError());
}

int launch_compact(const JoinQ* d_jobs, const int64_t* d_tile_base, int32_t njobs, int64_t total_tiles,
                   const uint2* d_pairs, const uint32_t* d_pair_uid, const int64_t* d_tile_src,
                   const int32_t* d_tile_cnt, const int64_t* d_tile_off, const BandOrder& bo, bool chain, void* st,
                   int sum) {
  if (total_tiles <= 0) return 0;
  const int2* perm = bo.key && bo.tile_job ? bo.perm : nullptr;
  if (sum != 1) {  // jobs without normalisation pieces (all of them when sum == 0)
    auto kc = chain ? k_compact<true> : k_compact<false>;
    hipLaunchKernelGGL(kc, dim3((unsigned)((total_tiles + COMPACT_TILES - 1) / COMPACT_TILES)), dim3(256), 0, S(st),
                       d_jobs, d_tile_base, njobs, total_tiles, d_pairs, d_pair_uid, d_tile_src, d_tile_cnt, d_tile_off,
                       perm, (const int32_t*)bo.tile_job, sum ? 1 : 0);
  }
  if (sum) {  // the jobs with pieces: one wave per tile
    auto ks = chain ? k_compact_sum<true> : k_compact_sum<false>;
    hipLaunchKernelGGL(ks, dim3((unsigned)total_tiles), dim3(64), 0, S(st), d_jobs, d_tile_base, njobs, total_tiles,
                       d_pairs, d_pair_uid, d_tile_src, d_tile_cnt, d_tile_off, perm, (const int32_t*)bo.tile_job);
  }
  return rc(hipGetLastError());
}

static inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

int launch_host_count(const uint64_t* hkeys, int64_t nslots, int world, uint32_t* owner_cnt, void* st,
                      const uint64_t* host_key) {
  if (nslots > 0)
    hipLaunchKernelGGL(k_host_count, dim3(nblk(nslots)), dim3(256), 0, S(st), hkeys, nslots, world, owner_cnt, host_key);
  return rc(hipGetLastError());
}

int launch_host_pack(const uint64_t* hkeys, const uint32_t* hcnt, const int64_t* slot_base, int nq, int64_t nslots,
                     int world, uint32_t* cursor, HostMsg* send, uint64_t* send_slot, void* st,
                     const uint64_t* host_key) {
  if (nslots > 0)
    hipLaunchKernelGGL(k_host_pack, dim3(nblk(nslots)), dim3(256), 0, S(st), hkeys, hcnt, slot_base, nq, nslots, world,
                       cursor, send, send_slot, host_key);
  return rc(hipGetLastError());
}

int launch_host_owner(const HostMsg* recv, int64_t nrecv, uint64_t* okeys, uint32_t* ocnt, uint64_t omask,
                      int32_t* gmax, uint32_t* reply, void* st) {
  if (nrecv > 0) {
    hipLaunchKernelGGL(k_host_insert, dim3(nblk(nrecv)), dim3(256), 0, S(st), recv, nrecv, okeys, ocnt, omask);
    hipLaunchKernelGGL(k_host_max, dim3(nblk((int64_t)omask + 1)), dim3(256), 0, S(st), okeys, ocnt,
                       (int64_t)omask + 1, gmax);
    hipLaunchKernelGGL(k_host_reply, dim3(nblk(nrecv)), dim3(256), 0, S(st), recv, nrecv, okeys, ocnt, omask, reply);
  }
  return rc(hipGetLastError());
}

int launch_host_apply(const uint32_t* back, const uint64_t* send_slot, int64_t n, uint32_t* hcnt_all, ShardSum* ss,
                      const int32_t* gmax, int nq, void* st) {
  if (n > 0) hipLaunchKernelGGL(k_host_apply, dim3(nblk(n)), dim3(256), 0, S(st), back, send_slot, n, hcnt_all);
  hipLaunchKernelGGL(k_set_maxdom, dim3(nblk(nq)), dim3(256), 0, S(st), ss, gmax, nq);
  return rc(hipGetLastError());
}

#ifdef YRWI_CHAIN_PROF
extern "C" int yrwi_chain_prof(unsigned long long* out) {  // profiling build only: read and clear
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cprof), sizeof(g_cprof)) != hipSuccess) return -1;
  unsigned long long z[24] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_cprof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

int launch_reduce(const RankQ* d_q, const int64_t* d_chunk_base, const int32_t* d_chunk_q, int32_t nq,
                  int64_t total_chunks,
                  ChunkSum* d_chunks, ShardSum* d_shard, void* st, void* ev_mid, bool hp_any, bool reduce,
                  const int2* d_group_q, int64_t ngroups) {
  // (static, the 4 KB cost every batch's k_reduce LDS whether it counted hosts or not)
  if (total_chunks > 0 && reduce)
    hipLaunchKernelGGL(k_reduce, dim3((unsigned)total_chunks), dim3(CHUNK_THREADS),
                       hp_any ? HPART_MAXS * sizeof(int32_t) : 0, S(st), d_q, d_chunk_q, d_chunks, d_shard);
  if (ngroups > 0) hipLaunchKernelGGL(k_piece_merge, dim3((unsigned)ngroups), dim3(64), 0, S(st), d_q, d_group_q);
  if (ev_mid) hipEventRecord(reinterpret_cast<hipEvent_t>(ev_mid), S(st));  // k_reduce alone (statistics)
  hipLaunchKernelGGL(k_shard_fin, dim3((unsigned)nq), dim3(64), 0, S(st), d_q, d_chunk_base, d_chunks, d_shard);
  return rc(hipGetLastError());
}

int launch_host_part(const RankQ* d_q, const int32_t* d_chunk_q, int64_t total_chunks, int32_t* d_hist,
                     int32_t* d_hoffs, int64_t nhist, void* d_tmp, size_t tmp_bytes, uint2* d_part, const int2* d_bq,
                     int32_t nbuckets, ShardSum* d_shard, void* st) {
  if (total_chunks <= 0 || nbuckets <= 0) return 0;
  // (the histogram: k_reduce, launched before on this stream)
  size_t t = tmp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(d_tmp, t, d_hist, d_hoffs, (int)(nhist + 1), S(st)) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_hpart_scatter, dim3((unsigned)total_chunks), dim3(CHUNK_THREADS), 0, S(st), d_q, d_chunk_q,
                     (const int32_t*)d_hoffs, d_part);
  hipLaunchKernelGGL(k_hbucket, dim3((unsigned)nbuckets), dim3(CHUNK_THREADS), 0, S(st), d_q, d_bq,
                     (const int32_t*)d_hoffs, (const uint2*)d_part, d_shard);
  return rc(hipGetLastError());
}

size_t host_part_tmp_bytes(int64_t nhist) {
  size_t t = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, t, (int32_t*)nullptr, (int32_t*)nullptr, (int)(nhist + 1), (hipStream_t)0);
  return t;
}

int launch_combine(const RankQ* d_q, int32_t nq, const ShardSum* d_shards, int32_t world, NormState* d_norm,
                   void* st) {
  hipLaunchKernelGGL(k_combine, dim3((unsigned)((nq + 63) / 64)), dim3(64), 0, S(st), d_q, nq, d_shards, world, d_norm);
  return rc(hipGetLastError());
}

int launch_score(const RankQ* d_q, const int32_t* d_chunk_q, const int32_t* d_order, int32_t nq, int64_t total_chunks,
                 int64_t seed_chunks, const NormState* d_norm, Cand* d_cand, int32_t* d_cand_cnt, int32_t kc,
                 int32_t* d_redo, int32_t* d_nredo, unsigned long long* d_tq, void* d_qtab, void* st,
                 void* ev_mid) {
  if (total_chunks <= 0) {  // (the statistics' event is recorded all the same: its elapsed time is read)
    if (ev_mid) hipEventRecord(reinterpret_cast<hipEvent_t>(ev_mid), S(st));
    return 0;
  }
  QTab* qt = reinterpret_cast<QTab*>(d_qtab);
  hipLaunchKernelGGL(k_qtabs, dim3((unsigned)nq), dim3(256), 0, S(st), d_q, d_norm, qt);
  // seed_chunks (0 < seed < total): the first chunks of `order` run as a launch of
  // their own, so every later chunk starts with its query's threshold set
  const int64_t s0 = (seed_chunks > 0 && seed_chunks < total_chunks) ? seed_chunks : total_chunks;
  hipLaunchKernelGGL(k_score, dim3((unsigned)s0), dim3(CHUNK_THREADS), 0, S(st), d_q, d_chunk_q, d_order, d_norm,
                     d_cand, d_cand_cnt, kc, d_redo, d_nredo, d_tq, (const QTab*)qt);
  if (s0 < total_chunks)
    hipLaunchKernelGGL(k_score, dim3((unsigned)(total_chunks - s0)), dim3(CHUNK_THREADS), 0, S(st), d_q, d_chunk_q,
                       d_order + 2 * s0, d_norm, d_cand, d_cand_cnt, kc, d_redo, d_nredo, d_tq, (const QTab*)qt);
  if (ev_mid) hipEventRecord(reinterpret_cast<hipEvent_t>(ev_mid), S(st));  // the k_score launches alone (statistics)
  const unsigned g = (unsigned)std::min<int64_t>(total_chunks, 512);
  hipLaunchKernelGGL(k_score_full, dim3(g), dim3(CHUNK_THREADS), 0, S(st), d_q, d_chunk_q, d_norm, d_cand,
                     d_cand_cnt, kc, d_redo, d_nredo);
#ifdef YRWI_PHASE_CLOCK
  {
    static std::vector<unsigned long long> h;
    const int nb = (int)std::min<int64_t>(total_chunks, PH_MAXB);
    h.assign((size_t)nb * 8, 0);
    hipStreamSynchronize(S(st));
    hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_ts), h.size() * 8);
    // stamps: 0 start, 6 prologue, 1 score, 2 threshold, 3 scatter, 4 sort, 5 take (0: block left earlier)
    const int ord[7] = {0, 6, 1, 2, 3, 4, 5};
    double dur[7] = {0}, cnt[7] = {0}, life = 0;
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int b = 0; b < nb; b++) {
      const unsigned long long* x = &h[(size_t)b * 8];
      unsigned long long prev = x[0], last = x[0];
      t0 = std::min(t0, x[0]);
      for (int j = 1; j < 7; j++) {
        const unsigned long long v = x[ord[j]];
        if (!v || v < prev) break;
        dur[j] += (double)(v - prev);
        cnt[j] += 1;
        prev = last = v;
      }
      t1 = std::max(t1, last);
      life += (double)(last - x[0]);
    }
    fprintf(stderr, "PHASE span %.1f us, mean block life %.2f us, mean concurrency %.0f; per block us (n):", (t1 - t0) / 100.0,
            life / nb / 100.0, life / (double)(t1 - t0));
    const char* nm[7] = {"", "pro", "score", "thr", "scat", "sort", "take"};
    for (int j = 1; j < 7; j++) fprintf(stderr, " %s %.2f (%.0f)", nm[j], cnt[j] ? dur[j] / cnt[j] / 100.0 : 0.0, cnt[j]);
    fprintf(stderr, "\n");
    unsigned long long g[16];
    hipMemcpyFromSymbol(g, HIP_SYMBOL(g_phase), sizeof(g));
    fprintf(stderr, "PRUNE elems %llu survive %llu waves %llu all-pruned %llu\n", g[0], g[1], g[2], g[3]);
    for (auto& x : g) x = 0;
    hipMemcpyToSymbol(HIP_SYMBOL(g_phase), g, sizeof(g));
    std::vector<unsigned long long> z(h.size(), 0);
    hipMemcpyToSymbol(HIP_SYMBOL(g_ts), z.data(), z.size() * 8);
  }
#endif
  return rc(hipGetLastError());
}

int topq_capacity(int32_t keff) { return keff <= 2048 ? 4096 : 8192; }
size_t score_qtab_bytes() { return sizeof(QTab); }

int launch_topq(const int64_t* d_gbase, const int32_t* d_gn, const int32_t* d_gk, int64_t ngroups, const Cand* d_in,
                const int32_t* d_in_cnt, int32_t in_stride, int32_t keff, Cand* d_out, int32_t* d_out_cnt, void* st) {
  if (ngroups <= 0) return 0;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_topq<4096>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * 4096 * sizeof(uint64_t)) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&k_topq<8192>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * 8192 * sizeof(uint64_t)) != hipSuccess)
      return YRWI_E_HIP;
    attr = true;
  }
  if (topq_capacity(keff) == 4096)
    hipLaunchKernelGGL(k_topq<4096>, dim3((unsigned)ngroups), dim3(TOPQ_THREADS), 2 * 4096 * sizeof(uint64_t), S(st),
                       d_gbase, d_gn, d_gk, d_in, d_in_cnt, in_stride, keff, d_out, d_out_cnt);
  else
    hipLaunchKernelGGL(k_topq<8192>, dim3((unsigned)ngroups), dim3(TOPQ_THREADS), 2 * 8192 * sizeof(uint64_t), S(st),
                       d_gbase, d_gn, d_gk, d_in, d_in_cnt, in_stride, keff, d_out, d_out_cnt);
  return rc(hipGetLastError());
}

// ReferenceOrder.cardinal(URIMetadataNode) (ReferenceOrder.java:267-296): all
// terms are Java ints, summed with int wrap, then widened.  lang: the order's
// language (8 bytes, NUL padded); a node language equal to it as a string scores.
__global__ void k_score_nodes(const yrwi_node* __restrict__ nodes, int64_t n, const yrwi_profile* __restrict__ prof,
                              uint64_t lang, int32_t maxdomcount, int64_t* __restrict__ scores) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const yrwi_node& t = nodes[i];
  const yrwi_profile& rk = *prof;
  const uint32_t z = t.flags[0] | ((uint32_t)t.flags[1] << 8) | ((uint32_t)t.flags[2] << 16) |
                     ((uint32_t)t.flags[3] << 24);
  const int dl = ahpla(t.urlhash[11]) & 3;
  const int32_t dln = dl == 0 ? 4 : dl == 1 ? 10 : dl == 2 ? 14 : 20;  // << (8/20) == << 0
  int32_t r = shl32(256 - dln, rk.coeff_domlength);
  r = add32(r, shl32(t.virtual_age, rk.coeff_date));
  r = add32(r, shl32(t.wordsintitle, rk.coeff_wordsintitle));
  r = add32(r, shl32(t.wordcount, rk.coeff_wordsintext));
  r = add32(r, shl32(t.llocal, rk.coeff_llocal));
  r = add32(r, shl32(t.lother, rk.coeff_lother));
  if (rk.coeff_authority > 12)
    r = add32(r, shl32(div32(shl32(t.host_count, 8), add32(1, maxdomcount)), rk.coeff_authority));
  const int32_t c255 = 255;
  if (z & (1u << 28)) r = add32(r, shl32(c255, rk.coeff_appurl));
  if (z & (1u << 25)) r = add32(r, shl32(c255, rk.coeff_app_dc_title));
  if (z & (1u << 26)) r = add32(r, shl32(c255, rk.coeff_app_dc_creator));
  if (z & (1u << 27)) r = add32(r, shl32(c255, rk.coeff_app_dc_subject));
  if (z & (1u << 24)) r = add32(r, shl32(c255, rk.coeff_app_dc_description));
  if (z & (1u << 29)) r = add32(r, shl32(c255, rk.coeff_appemph));
  if (z & (1u << 0)) r = add32(r, shl32(c255, rk.coeff_catindexof));
  if (z & (1u << 20)) r = add32(r, shl32(c255, rk.coeff_cathasimage));
  if (z & (1u << 21)) r = add32(r, shl32(c255, rk.coeff_cathasaudio));
  if (z & (1u << 22)) r = add32(r, shl32(c255, rk.coeff_cathasvideo));
  if (z & (1u << 23)) r = add32(r, shl32(c255, rk.coeff_cathasapp));
  uint64_t nl = 0;
  for (int j = 0; j < 8; j++) nl |= (uint64_t)(uint8_t)t.language[j] << (8 * j);
  if (nl != 0 && nl == lang) r = add32(r, shl32(c255, rk.coeff_language));
  scores[i] = (int64_t)r;
}

int launch_score_nodes(const yrwi_node* d_nodes, int64_t n, const yrwi_profile* d_prof, const char* lang8,
                       int32_t maxdomcount, int64_t* d_scores, void* st) {
  if (n <= 0) return 0;
  uint64_t lang = 0;
  for (int j = 0; j < 8 && lang8[j]; j++) lang |= (uint64_t)(uint8_t)lang8[j] << (8 * j);
  hipLaunchKernelGGL(k_score_nodes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), d_nodes, n, d_prof, lang,
                     maxdomcount, d_scores);
  return rc(hipGetLastError());
}

__global__ void k_reduce_i32(const int32_t* __restrict__ all, int world, int64_t n, int32_t* __restrict__ out,
                             int max_op) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t v = all[i];
  for (int r = 1; r < world; r++) {
    const int32_t x = all[(int64_t)r * n + i];
    v = max_op ? (x > v ? x : v) : (int32_t)((uint32_t)v + (uint32_t)x);
  }
  out[i] = v;
}

int launch_reduce_i32(const int32_t* all, int world, int64_t n, int32_t* out, int max_op, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_reduce_i32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), all, world, n, out, max_op);
  return rc(hipGetLastError());
}

int launch_pull(const RankQ* d_q, int32_t nq, const yrwi_hit* d_stack, const int32_t* d_scnt, int32_t kint,
                int only_dd, int32_t kmax, yrwi_hit* d_hits, int32_t* d_nout, void* st) {
  if (nq <= 0) return 0;
  hipLaunchKernelGGL(k_pull, dim3((unsigned)nq), dim3(64), 0, S(st), d_q, d_stack, d_scnt, kint, only_dd, kmax, d_hits,
                     d_nout);
  return rc(hipGetLastError());
}

int launch_gmerge(const RankQ* d_q, const yrwi_hit* d_allh, const int32_t* d_alln, int world, int32_t nq, int32_t kint,
                  uint32_t* d_slot, uint8_t* d_dup, yrwi_hit* d_stack, int32_t* d_scnt, void* st) {
  if (nq <= 0) return 0;
  const int64_t n = (int64_t)nq * world * kint;
  hipLaunchKernelGGL(k_gmerge_rank, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), d_allh, d_alln, world, nq,
                     kint, d_slot, d_dup);
  hipLaunchKernelGGL(k_gmerge_out, dim3((unsigned)nq), dim3(256), 0, S(st), d_q, d_allh, d_alln, world, nq, kint, d_slot,
                     d_dup, d_stack, d_scnt);
  return rc(hipGetLastError());
}

int launch_emit(const RankQ* d_q, int32_t nq, const Cand* const* d_final, const int32_t* const* d_final_cnt,
                int32_t kmax, yrwi_hit* d_hits, int32_t* d_nout, int mode, void* st) {
  hipLaunchKernelGGL(k_emit, dim3((unsigned)nq), dim3(256), 0, S(st), d_q, nq, d_final, d_final_cnt, kmax,
                     d_hits, d_nout, mode);
  return rc(hipGetLastError());
}

int launch_score_all(const RankQ* d_q, const int32_t* d_chunk_q, int32_t nq, int64_t total_chunks,
                     const NormState* d_norm, int64_t* d_scores, void* st) {
  if (total_chunks <= 0) return 0;
  hipLaunchKernelGGL(k_score_all, dim3((unsigned)total_chunks), dim3(256), 0, S(st), d_q, d_chunk_q, d_norm,
                     d_scores);
  return rc(hipGetLastError());
}

// ======================================= search events
// SearchEvent.addRWIs (SearchEvent.java:673-836) applied to one container after
// another -- the local RWI process and every remote peer's result
// (Protocol.remoteSearchProcess :670-830 -> addRWIs(local=false) :802).  The
// per-arrival semantics: normalizeWith continues the event's ReferenceOrder
// (min/max, max-distance fold, host counts; settled over the arrival before it
// is scored, as the local path), the doublecheck set, the flag counts and the
// bounded rwiStack carry over; entries already on the stack keep the score they
// were given on arrival.  One workgroup owns an event for a launch and applies
// its arrivals in order, so all event state is touched by one workgroup only.

__device__ __forceinline__ uint64_t ld_dev(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_dev32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Url set of 72-bit url keys with 64-bit CAS: 9 key bits (XOR-mixed with the
// other 63, a bijection) choose one of EV_SUBS sub-tables and the other 63 bits
// plus an occupied bit are the stored word, so equal words in one sub-table are
// equal keys and an insert is one compare-and-swap.
__device__ __forceinline__ void uset_slot(uint64_t hi, uint32_t lo, int ulog, uint64_t& word, int64_t& base,
                                          uint32_t& start) {
  const uint64_t h63 = hi >> 1;
  const uint32_t b9 = ((uint32_t)(hi & 1u) << 8) | (lo & 0xFFu);
  const uint64_t m = mix64(h63);
  base = (int64_t)((b9 ^ (uint32_t)m) & (uint32_t)(EV_SUBS - 1)) << ulog;
  start = (uint32_t)(m >> 32);
  word = h63 | (1ull << 63);
}
__device__ int64_t uset_insert(uint64_t* key, int ulog, uint64_t hi, uint32_t lo) {
  uint64_t w;
  int64_t base;
  uint32_t st;
  uset_slot(hi, lo, ulog, w, base, st);
  const uint32_t mask = (1u << ulog) - 1;
  for (uint32_t t = 0; t <= mask; t++) {
    const int64_t s = base + ((st + t) & mask);
    const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(key + s), 0ull, (unsigned long long)w);
    if (prev == 0 || prev == w) return s;
  }
  return -1;
}
__device__ int64_t uset_find(const uint64_t* key, int ulog, uint64_t hi, uint32_t lo) {
  uint64_t w;
  int64_t base;
  uint32_t st;
  uset_slot(hi, lo, ulog, w, base, st);
  const uint32_t mask = (1u << ulog) - 1;
  for (uint32_t t = 0; t <= mask; t++) {
    const int64_t s = base + ((st + t) & mask);
    const uint64_t k = ld_dev(key + s);
    if (k == w) return s;
    if (k == 0) return -1;
  }
  return -1;
}

// event host counts (ReferenceOrder.doms, ConcurrentScoreMap.inc :184): keys host36 + 1
__device__ int64_t htab_insert(uint64_t* keys, uint64_t mask, uint64_t key) {
  uint64_t s = mix64(key) & mask;
  for (uint64_t t = 0; t <= mask; t++) {
    const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(keys + s), 0ull, (unsigned long long)key);
    if (prev == 0 || prev == key) return (int64_t)s;
    s = (s + 1) & mask;
  }
  return -1;
}
__device__ int32_t htab_count(const uint64_t* keys, const uint32_t* cnt, uint64_t mask, uint64_t key) {
  uint64_t s = mix64(key) & mask;
  for (uint64_t t = 0; t <= mask; t++) {
    const uint64_t k = ld_dev(keys + s);
    if (k == key) return (int32_t)ld_dev32(cnt + s);
    if (k == 0) return 0;
    s = (s + 1) & mask;
  }
  return 0;
}

__global__ void k_event_seed(const EvDev* __restrict__ ev, const uint64_t* __restrict__ hi,
                             const uint8_t* __restrict__ lo, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s = uset_insert(ev->ukey, ev->ulog, hi[i], lo[i]);
  if (s < 0) atomicExch(&ev->st->err, (int32_t)YRWI_E_CAPACITY);
  else atomicMin(reinterpret_cast<unsigned long long*>(ev->uval + s), 0ull);  // epoch 0: in urlhashes from the start
}

__global__ __launch_bounds__(EV_THREADS) void k_event_add(const EvDev* __restrict__ evs,
                                                          const EvJob* __restrict__ jobs,
                                                          const int32_t* __restrict__ jb,
                                                          int32_t* __restrict__ status) {
  __shared__ EvState S;
  __shared__ NormState N;
  __shared__ int32_t sP[EV_CH], sO[EV_CH];
  __shared__ uint64_t sK1[EV_CH], sK2[EV_CH];
  __shared__ Cand sC[EV_CH];
  __shared__ int32_t sKeep[EV_CH + 1];
  __shared__ int32_t sSegM[65], sSegL[65], sSegP[65];
  __shared__ int32_t sFlag[32];
  __shared__ int32_t sRedI[EV_THREADS / 64][2 * NF + 2];
  __shared__ double sRedD[EV_THREADS / 64][2];
  __shared__ int32_t sScan[16];
  __shared__ int32_t sMisc[8];  // 0 validation bits, 1 candidates, 2 admitted, 3 max host count, 4 overflow
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j0 = jb[blockIdx.x], j1 = jb[blockIdx.x + 1];
  const EvDev& E = evs[jobs[j0].ev];
  const RankQ& Q = E.q;
  const int32_t K = Q.k;
  if (tid == 0) S = *E.st;
  __syncthreads();
  for (int j = j0; j < j1; j++) {
    const EvJob J = jobs[j];
    const int64_t n = J.n;
    if (S.err || n <= 0) {
      if (tid == 0) status[j] = S.err;
      continue;
    }
    const uint8_t* rows = J.rows;
    if (tid < 8) sMisc[tid] = 0;
    __syncthreads();
    // ---- validation: Base64 url hashes, a language cell (the reference NPEs on 0x0000)
    {
      int bad = 0;
      for (int64_t i = tid; i < n; i += EV_THREADS) {
        const Row R = load_row(rows + i * YRWI_ROW_BYTES);
        for (int q = 0; q < 12; q++) bad |= ahpla(R.b(q)) < 0 ? 1 : 0;
        if (R.b(O_L) == 0 && R.b(O_L + 1) == 0) bad |= 2;
      }
      if (bad) atomicOr(&sMisc[0], bad);
      __syncthreads();
      const int verr = sMisc[0];
      if (verr) {
        if (tid == 0) status[j] = (verr & 1) ? YRWI_E_HASH : YRWI_E_NULL_LANGUAGE;
        __syncthreads();
        continue;
      }
    }
    // ---- normalizeWith over the arrival, continuing the event's min/max (:163-210)
    const bool first = !S.started;
    int32_t mn[NF], mx[NF], vmn = BIG, vmx = -1;
    double tmn = 1e300, tmx = -1e300;
    for (int f = 0; f < NF; f++) { mn[f] = BIG; mx[f] = -1; }
    int32_t fP = S.P, fA = S.A;
    int fH = S.hasA;
    for (int64_t c0 = 0; c0 < n; c0 += EV_CH) {
      const int m = (int)min((int64_t)EV_CH, n - c0);
      for (int s = 0; s < EV_CH / EV_THREADS; s++) {
        const int li = s * EV_THREADS + tid;
        if (li >= m) break;
        const Row R = load_row(rows + (c0 + li) * YRWI_ROW_BYTES);
        const Feat t = decode(R);
        int32_t a = t.a, od = t.od;
        if (first && c0 == 0 && li == 0) { a = clamp_days(a, Q.now_ms); od = 0; }  // the clone (:357-361)
        for (int f = 0; f < NF; f++) { mn[f] = min(mn[f], t.f[f]); mx[f] = max(mx[f], t.f[f]); }
        vmn = min(vmn, a);
        vmx = max(vmx, a);
        tmn = fmin(tmn, t.tf);
        tmx = fmax(tmx, t.tf);
        sP[li] = t.p;
        sO[li] = od;
      }
      __syncthreads();
      if (wv == 0) {  // the order-dependent max-distance fold, 64 elements a round
        if (first && c0 == 0) { fP = sP[0]; fA = 0; fH = 0; }
        for (int base = 0; base < m; base += 64) {
          const int i = base + lane;
          const bool v = i < m;
          const int32_t p = v ? sP[i] : 0, od = v ? sO[i] : 0;
          const int32_t Pi = max(fP, wave_incl_max(p));
          int32_t Pprev = __shfl_up(Pi, 1, 64);
          if (lane == 0) Pprev = fP;
          const bool rec = v && Pi > Pprev;  // a new running maximum of posintext starts a segment
          const uint64_t rm = __ballot(rec);
          const int seg = __popcll(rm & (lane == 63 ? ~0ull : ((2ull << lane) - 1)));
          sSegM[lane] = 0;
          sSegL[lane] = -1;
          if (lane == 0) { sSegM[64] = 0; sSegL[64] = -1; }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          if (rec) sSegP[seg] = Pi;
          if (v) {
            atomicMax(&sSegM[seg], od);
            if (od > 0) atomicMax(&sSegL[seg], lane);
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          const int nseg = __popcll(rm);
          if (lane == 0) {
            Fold fd{fP, fA, fH != 0};
            for (int sg = 0; sg <= nseg; sg++) {
              const int32_t Ls = sSegL[sg];
              fd.piece(sg == 0 ? fP : sSegP[sg], sSegM[sg], Ls >= 0 ? sO[base + Ls] : 0);
            }
            fP = fd.P;
            fA = fd.A;
            fH = fd.hasA ? 1 : 0;
          }
          fP = __shfl(fP, 0, 64);
          fA = __shfl(fA, 0, 64);
          fH = __shfl(fH, 0, 64);
          __builtin_amdgcn_wave_barrier();
        }
      }
      __syncthreads();
    }
    for (int f = 0; f < NF; f++) {
      const int32_t a = wave_min_i(mn[f]), b = wave_max_i(mx[f]);
      if (lane == 0) { sRedI[wv][f] = a; sRedI[wv][NF + f] = b; }
    }
    {
      const int32_t a = wave_min_i(vmn), b = wave_max_i(vmx);
      const double c = wave_min_d(tmn), d = wave_max_d(tmx);
      if (lane == 0) { sRedI[wv][2 * NF] = a; sRedI[wv][2 * NF + 1] = b; sRedD[wv][0] = c; sRedD[wv][1] = d; }
    }
    __syncthreads();
    if (tid == 0) {
      for (int w = 0; w < EV_THREADS / 64; w++) {
        for (int f = 0; f < NF; f++) {
          S.mn[f] = (first && w == 0) ? sRedI[w][f] : min(S.mn[f], sRedI[w][f]);
          S.mx[f] = (first && w == 0) ? sRedI[w][NF + f] : max(S.mx[f], sRedI[w][NF + f]);
        }
        S.va_mn = (first && w == 0) ? sRedI[w][2 * NF] : min(S.va_mn, sRedI[w][2 * NF]);
        S.va_mx = (first && w == 0) ? sRedI[w][2 * NF + 1] : max(S.va_mx, sRedI[w][2 * NF + 1]);
        S.tf_mn = (first && w == 0) ? sRedD[w][0] : fmin(S.tf_mn, sRedD[w][0]);
        S.tf_mx = (first && w == 0) ? sRedD[w][1] : fmax(S.tf_mx, sRedD[w][1]);
      }
      S.P = fP;
      S.A = fA;
      S.hasA = fH;
      S.started = 1;
    }
    // ---- host counts (doms, maxdomcount; only read by authority)
    if (Q.want_authority) {
      int32_t hm = 0, ovf = 0;
      for (int64_t i = tid; i < n; i += EV_THREADS) {
        const Row R = load_row(rows + i * YRWI_ROW_BYTES);
        const int64_t s = htab_insert(Q.hkeys, Q.hmask, host36(R) + 1);
        if (s < 0) ovf = 1;
        else hm = max(hm, (int32_t)atomicAdd(Q.hcnt + s, 1u) + 1);
      }
      hm = wave_max_i(hm);
      if (lane == 0 && hm) atomicMax(&sMisc[3], hm);
      if (ovf) atomicOr(&sMisc[4], 1);
    }
    __syncthreads();
    if (tid == 0) {
      S.maxdom = max(S.maxdom, sMisc[3]);
      for (int f = 0; f < NF; f++) { N.mn[f] = S.mn[f]; N.mx[f] = S.mx[f]; }
      N.va_mn = S.va_mn;
      N.va_mx = S.va_mx;
      N.tf_mn = S.tf_mn;
      N.tf_mx = S.tf_mx;
      N.maxdom = S.maxdom;
      N.nvalid = 1;
      Fold fd{S.P, S.A, S.hasA != 0};
      N.D = fd.D();
      for (int f = 0; f < NF; f++) N.rcp[f] = N.mx[f] != N.mn[f] ? 1.0 / (double)(N.mx[f] - N.mn[f]) : 0.0;
      N.rcp[NF] = N.va_mx != N.va_mn ? 1.0 / (double)(N.va_mx - N.va_mn) : 0.0;
      N.rcp[NF + 1] = N.D != 0 ? 1.0 / (double)N.D : 0.0;
    }
    if (J.scores) {  // yrwi_event_order: cardinal of every row under the state after this container
      __syncthreads();
      if (sMisc[4]) {
        if (tid == 0) { S.err = YRWI_E_CAPACITY; status[j] = YRWI_E_CAPACITY; }
        __syncthreads();
        continue;
      }
      for (int64_t i = tid; i < n; i += EV_THREADS) {
        const Row R = load_row(rows + i * YRWI_ROW_BYTES);
        const int32_t hc = Q.want_authority ? htab_count(Q.hkeys, Q.hcnt, Q.hmask, host36(R) + 1) : 0;
        J.scores[i] = cardinal(decode(R), N, Q, hc);
      }
      __syncthreads();
      if (tid == 0) {
        S.nin += n;
        status[j] = 0;
      }
      __syncthreads();
      continue;
    }
    // ---- doublecheck: the first occurrence of a url passing the constraints is admitted (:736-805)
    const uint32_t ep = (uint32_t)S.epoch + 1;
    {
      int ovf = 0;
      for (int64_t i = tid; i < n; i += EV_THREADS) {
        const Row R = load_row(rows + i * YRWI_ROW_BYTES);
        if (E.has_filter && !passes(E.f, decode(R), host36(R))) continue;
        uint64_t hi;
        uint32_t lo;
        row_key(R, hi, lo);
        const int64_t s = uset_insert(E.ukey, E.ulog, hi, lo);
        if (s < 0) { ovf = 1; continue; }
        atomicMin(reinterpret_cast<unsigned long long*>(E.uval + s), ((uint64_t)ep << 32) | (uint64_t)i);
      }
      if (ovf) atomicOr(&sMisc[4], 1);
    }
    __threadfence();
    __syncthreads();
    if (sMisc[4]) {  // a table is full: the event is unusable (max_postings too small)
      if (tid == 0) { S.err = YRWI_E_CAPACITY; status[j] = YRWI_E_CAPACITY; }
      __syncthreads();
      continue;
    }
    // ---- flag counts, cardinal, rwiStack.put per chunk
    if (tid < 32) sFlag[tid] = 0;
    int32_t nadm = 0;
    for (int64_t c0 = 0; c0 < n; c0 += EV_CH) {
      const int m = (int)min((int64_t)EV_CH, n - c0);
      if (tid == 0) sMisc[1] = 0;
      __syncthreads();
      for (int s = 0; s < EV_CH / EV_THREADS; s++) {
        const int li = s * EV_THREADS + tid;
        if (li >= m) break;
        const int64_t i = c0 + li;
        const Row R = load_row(rows + i * YRWI_ROW_BYTES);
        uint64_t hi;
        uint32_t lo;
        row_key(R, hi, lo);
        const int64_t idx = uset_find(E.ukey, E.ulog, hi, lo);
        const uint64_t v = idx >= 0 ? ld_dev(E.uval + idx) : ~0ull;
        if (idx >= 0 && (uint32_t)(v >> 32) < ep) continue;  // already in urlhashes: dropped uncounted
        const bool found = idx >= 0;
        const uint32_t fi = found ? (uint32_t)v : 0xFFFFFFFFu;
        if (!found || (uint32_t)i <= fi) {  // reaches the flag count (later duplicates hit the doublecheck)
          const uint32_t z = (R.b(O_Z) | (R.b(O_Z + 1) << 8) | (R.b(O_Z + 2) << 16) | (R.b(O_Z + 3) << 24));
          for (uint32_t mm = z; mm; mm &= mm - 1) atomicAdd(&sFlag[__ffs(mm) - 1], 1);  // (flagcount :743-746)
        }
        if (found && (uint32_t)i == fi) {
          const Feat t = decode(R);
          const int32_t hc = Q.want_authority ? htab_count(Q.hkeys, Q.hcnt, Q.hmask, host36(R) + 1) : 0;
          const int64_t sc = cardinal(t, N, Q, hc);
          const int slot = atomicAdd(&sMisc[1], 1);
          sK1[slot] = (uint64_t)sc ^ 0x8000000000000000ull;
          sK2[slot] = ((uint64_t)((uint32_t)url_hashcode(R) ^ 0x80000000u) << 32) | (uint64_t)(~(uint32_t)i);
          nadm++;
        }
      }
      __syncthreads();
      const int nc = sMisc[1];
      __syncthreads();  // every thread has nc before the next chunk resets it
      if (nc == 0) continue;
      const int NP = pow2_at_least(nc);
      for (int x = nc + tid; x < NP; x += EV_THREADS) { sK1[x] = 0; sK2[x] = 0; }
      __syncthreads();
      bitonic_desc<EV_THREADS>(sK1, sK2, NP);
      int32_t dist;
      const int32_t c = dedupe_take<EV_THREADS>(sK1, sK2, NP, K, sC, sScan, &dist);
      __syncthreads();
      // merge the chunk's TreeSet classes into the stack: an entry equal in
      // (score, hashCode) to one already there is rejected (it arrived later)
      const yrwi_hit* cur = E.stack + (int64_t)S.cur * K;
      yrwi_hit* nxt = E.stack + (int64_t)(S.cur ^ 1) * K;
      const int32_t ns = S.nstack;
      int32_t keep[EV_CH / EV_THREADS], pos[EV_CH / EV_THREADS], nk = 0;
      for (int q = 0; q < EV_CH / EV_THREADS; q++) {
        const int x = tid * (EV_CH / EV_THREADS) + q;
        keep[q] = 0;
        pos[q] = 0;
        if (x >= c) continue;
        const int64_t sc = (int64_t)(sC[x].k1 ^ 0x8000000000000000ull);
        const int32_t tb = (int32_t)((uint32_t)(sC[x].k2 >> 32) ^ 0x80000000u);
        int lo = 0, hi = ns;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const int64_t hs = cur[mid].score;
          const int32_t ht = cur[mid].tiebreak;
          if (hs > sc || (hs == sc && ht > tb)) lo = mid + 1; else hi = mid;
        }
        const bool dup = lo < ns && cur[lo].score == sc && cur[lo].tiebreak == tb;
        keep[q] = dup ? 0 : 1;
        pos[q] = lo;
        nk += keep[q];
      }
      int32_t tot;
      int32_t off = block_excl_sum<EV_THREADS>(nk, sScan, &tot);
      for (int q = 0; q < EV_CH / EV_THREADS; q++) {
        const int x = tid * (EV_CH / EV_THREADS) + q;
        if (x < c) sKeep[x] = off;
        if (keep[q]) {
          const int32_t o = off + pos[q];
          if (o < K) {
            yrwi_hit h;
            const uint32_t ai = ~(uint32_t)sC[x].k2;
            const uint8_t* rr = rows + (int64_t)ai * YRWI_ROW_BYTES;
            for (int b = 0; b < 12; b++) h.urlhash[b] = rr[b];
            h.tiebreak = (int32_t)((uint32_t)(sC[x].k2 >> 32) ^ 0x80000000u);
            h.score = (int64_t)(sC[x].k1 ^ 0x8000000000000000ull);
            nxt[o] = h;
          }
          off++;
        }
      }
      if (tid == 0) sKeep[c] = tot;
      __syncthreads();
      for (int y = tid; y < ns; y += EV_THREADS) {
        const yrwi_hit h = cur[y];
        int lo = 0, hi = c;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const int64_t cs = (int64_t)(sC[mid].k1 ^ 0x8000000000000000ull);
          const int32_t ct = (int32_t)((uint32_t)(sC[mid].k2 >> 32) ^ 0x80000000u);
          if (cs > h.score || (cs == h.score && ct > h.tiebreak)) lo = mid + 1; else hi = mid;
        }
        const int32_t o = y + sKeep[lo];
        if (o < K) nxt[o] = h;
      }
      __threadfence();
      __syncthreads();
      if (tid == 0) {
        S.nstack = min(K, ns + tot);
        S.cur ^= 1;
      }
      __syncthreads();
    }
    nadm = wave_sum_i(nadm);
    if (lane == 0 && nadm) atomicAdd(&sMisc[2], nadm);
    __syncthreads();
    if (tid < 32) S.flagcount[tid] += sFlag[tid];
    if (tid == 0) {
      S.epoch = (int32_t)ep;
      S.nin += n;
      if (J.local) S.nadmit_local += sMisc[2];
      else { S.nadmit_remote += sMisc[2]; S.nremote += 1; }
      status[j] = 0;
    }
    __syncthreads();
  }
  if (tid == 0) *E.st = S;
}

__global__ void k_event_authority(const EvDev* __restrict__ ev, const uint64_t* __restrict__ keys, int32_t n,
                                  int32_t* __restrict__ out) {
  const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const RankQ& Q = ev->q;
  const int32_t c = Q.want_authority ? htab_count(Q.hkeys, Q.hcnt, Q.hmask, keys[i]) : 0;
  out[i] = div32(shl32(c, 8), add32(1, ev->st->maxdom));  // (doms.get(h) << 8) / (1 + maxdomcount)
}

int launch_sel_lookup(const uint64_t* d_hi, const uint8_t* d_lo, int64_t n, const uint64_t* dkhi, const uint8_t* dklo,
                      int64_t nurls, uint32_t* d_uid, void* st) {
  if (n > 0)
    hipLaunchKernelGGL(k_sel_lookup, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), d_hi, d_lo, n, dkhi, dklo,
                       nurls, d_uid);
  return rc(hipGetLastError());
}
int launch_sel_count(const SelCount* d_jobs, int32_t njobs, void* st) {
  if (njobs > 0) hipLaunchKernelGGL(k_sel_count, dim3((unsigned)njobs), dim3(256), 0, S(st), d_jobs);
  return rc(hipGetLastError());
}
int launch_sel_pick(const SelPick* d_jobs, int32_t njobs, void* st) {
  if (njobs > 0) hipLaunchKernelGGL(k_sel_pick, dim3((unsigned)njobs), dim3(256), 0, S(st), d_jobs);
  return rc(hipGetLastError());
}

// where each url entered the event's doublecheck set (SearchEvent.urlhashes): the
// (arrival epoch << 32 | row) of its admitted posting, ~0 if the url is not in it
__global__ void k_event_where(const EvDev* __restrict__ ev, const uint64_t* __restrict__ hi,
                              const uint8_t* __restrict__ lo, int32_t n, uint64_t* __restrict__ out) {
  const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const int64_t s = uset_find(ev->ukey, ev->ulog, hi[i], lo[i]);
  out[i] = s >= 0 ? ld_dev(ev->uval + s) : ~0ull;
}

int launch_event_where(const EvDev* d_ev, const uint64_t* d_hi, const uint8_t* d_lo, int32_t n, uint64_t* d_out,
                       void* st) {
  if (n > 0) hipLaunchKernelGGL(k_event_where, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), d_ev, d_hi, d_lo,
                                n, d_out);
  return rc(hipGetLastError());
}

int launch_event_authority(const EvDev* d_ev, const uint64_t* d_keys, int32_t n, int32_t* d_out, void* st) {
  if (n > 0) hipLaunchKernelGGL(k_event_authority, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(st), d_ev, d_keys, n,
                                d_out);
  return rc(hipGetLastError());
}

int launch_event_add(const EvDev* d_ev, const EvJob* d_jobs, const int32_t* d_jb, int32_t nblocks, int32_t* d_status,
                     void* st) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(k_event_add, dim3((unsigned)nblocks), dim3(EV_THREADS), 0, S(st), d_ev, d_jobs, d_jb, d_status);
  return rc(hipGetLastError());
}

int launch_event_seed(const EvDev* d_ev, const uint64_t* d_hi, const uint8_t* d_lo, int64_t n, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_event_seed, dim3(nblk(n)), dim3(256), 0, S(st), d_ev, d_hi, d_lo, n);
  return rc(hipGetLastError());
}

}  // namespace yrwi
