// yrwi_abstract.hip -- index abstracts and the secondary-search join
// (SURVEY.md §8f row 3).
//
// Serving side: WordReferenceFactory.compressIndex (WordReferenceFactory.java:
// 75-117) over a stored posting list: "{host:url6url6...,host:...}", hosts in
// Java String order (raw bytes), the 6-character url prefixes of one host in
// container order.  On the device: the 48-bit raw host of every posting is
// radix-sorted stably with its position, segment heads are counted by a scan,
// and every posting writes its bytes at 8*g + 8 + 6*p (g = its host's rank,
// p = its sorted position) -- no host-side pass over the list.
//
// Asking side: decompressIndex (:125-155) of every abstract received,
// SecondarySearchSuperviser.addAbstract (:43-65), SetTools.joinConstructive
// (:76-116) over the words and prepareSecondarySearch / wordsFromPeer
// (:71-196).  Every abstract is parsed in parallel (one thread per segment
// start), the (url, word, abstract) triples are radix-sorted by url, word and
// arrival, and one thread per url resolves the per-word peer, the join and the
// words each peer is asked for.
#include <hipcub/hipcub.hpp>

#include "yrwi_host.h"

using namespace yrwi;

namespace {

unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }

// Java String order of Base64 characters: '-' < '0'-'9' < 'A'-'Z' < '_' < 'a'-'z'
__device__ __forceinline__ int acode(uint32_t c) {
  if (c == '-') return 0;
  if (c >= '0' && c <= '9') return 1 + (int)(c - '0');
  if (c >= 'A' && c <= 'Z') return 11 + (int)(c - 'A');
  if (c == '_') return 37;
  if (c >= 'a' && c <= 'z') return 38 + (int)(c - 'a');
  return -1;
}
__device__ __forceinline__ uint8_t achar(int code) {
  if (code == 0) return '-';
  if (code <= 10) return (uint8_t)('0' + code - 1);
  if (code <= 36) return (uint8_t)('A' + code - 11);
  if (code == 37) return '_';
  return (uint8_t)('a' + code - 38);
}

// ------------------------------------------------------------ compressIndex
__global__ void k_ca_keys(const uint8_t* __restrict__ rows, const uint64_t* __restrict__ khi,
                          const uint8_t* __restrict__ klo, int64_t n, const uint64_t* __restrict__ ehi,
                          const uint8_t* __restrict__ elo, int64_t ne, uint64_t* __restrict__ keys,
                          uint32_t* __restrict__ vals, unsigned long long* __restrict__ nexcl) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* r = rows + i * YRWI_ROW_BYTES;
  uint64_t k = 0;
  for (int j = 6; j < 12; j++) k = (k << 8) | r[j];
  if (ne > 0) {  // excludeContainer.getReference(urlhash) != null
    const uint64_t h = khi[i];
    const uint8_t l = klo[i];
    int64_t a = 0, b = ne;
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (ehi[m] < h || (ehi[m] == h && elo[m] < l)) a = m + 1; else b = m;
    }
    if (a < ne && ehi[a] == h && elo[a] == l) {
      k = 1ull << 48;  // sorts behind every host
      atomicAdd(nexcl, 1ull);
    }
  }
  keys[i] = k;
  vals[i] = (uint32_t)i;
}

__global__ void k_ca_heads(const uint64_t* __restrict__ keys, int64_t n, uint32_t* __restrict__ flag) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) flag[p] = (p == 0 || keys[p] != keys[p - 1]) ? 1u : 0u;
}

// posting at sorted position p of host rank g: url prefix at 8g + 8 + 6p; a
// host's first posting also writes ",host:" in front of it
__global__ void k_ca_write(const uint8_t* __restrict__ rows, const uint64_t* __restrict__ keys,
                           const uint32_t* __restrict__ vals, const uint32_t* __restrict__ g1, int64_t n,
                           uint8_t* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int64_t g = (int64_t)g1[p] - 1;
  const uint8_t* r = rows + (int64_t)vals[p] * YRWI_ROW_BYTES;
  const int64_t o = 8 * g + 8 + 6 * p;
  for (int j = 0; j < 6; j++) out[o + j] = r[j];
  if (p == 0 || keys[p] != keys[p - 1]) {
    const int64_t s = 1 + 8 * g + 6 * p;
    for (int j = 0; j < 6; j++) out[s + j] = r[6 + j];
    out[s + 6] = ':';
    if (g > 0) out[s - 1] = ',';
  }
  if (p == 0) out[0] = '{';
  if (p == n - 1) out[o + 6] = '}';
}

// ------------------------------------------------------ decompress + join
struct AbsDesc {
  int64_t off, len;      // text bytes [off, off + len)
  int32_t word, peer;    // word rank, peer rank (String order)
  int64_t first_bad;     // first segment start that ends the parse (decompressIndex's loop test)
  int32_t err, pad;
};

__device__ __forceinline__ int find_abs(const AbsDesc* A, int na, int64_t b) {
  int lo = 0, hi = na - 1;  // last abstract with off <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (A[mid].off <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// b is where decompressIndex looks for the next "host:": the body start or just after a ','
__device__ __forceinline__ bool seg_start(const uint8_t* t, const AbsDesc& D, int64_t b, int64_t& bend) {
  if (D.len < 2 || t[D.off] != '{' || t[D.off + D.len - 1] != '}') return false;  // not an abstract: empty map
  bend = D.off + D.len - 1;
  if (b < D.off + 1 || b > bend) return false;
  return b == D.off + 1 || t[b - 1] == ',';
}

__global__ void k_ss_bad(const uint8_t* __restrict__ t, int64_t nbytes, AbsDesc* __restrict__ A, int na) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nbytes) return;
  const int a = find_abs(A, na, b);
  int64_t bend;
  if (!seg_start(t, A[a], b, bend)) return;
  if (bend - b < 13 || t[b + 6] != ':')  // while (ci.length() >= 13 && ci.byteAt(6) == ':')
    atomicMin(reinterpret_cast<unsigned long long*>(&A[a].first_bad), (unsigned long long)b);
}

// A segment starting at b (parsed: before the abstract's first bad start):
// its url count, or 0; sets the abstract's error for a run the reference would
// misparse (not a multiple of 6 characters, or not Base64).
__device__ __forceinline__ int64_t seg_urls(const uint8_t* t, AbsDesc* A, int na, int64_t b, int& a) {
  a = find_abs(A, na, b);
  const AbsDesc& D = A[a];
  int64_t bend;
  if (!seg_start(t, D, b, bend) || b >= D.first_bad) return 0;
  bool bad = false;
  for (int j = 0; j < 6; j++) bad |= acode(t[b + j]) < 0;
  int64_t e = b + 7;
  while (e < bend && t[e] != ',') {
    bad |= acode(t[e]) < 0;
    e++;
  }
  const int64_t len = e - (b + 7);
  if (bad || len % 6) {
    atomicOr(&A[a].err, 1);
    return 0;
  }
  return len / 6;
}

// SS_BYTES text positions per thread: count the urls of the segments starting
// there, reserve the block's output with one atomic, then write the (url key,
// word, abstract) triples
constexpr int SS_BYTES = 16;
__global__ __launch_bounds__(256) void k_ss_parse(const uint8_t* __restrict__ t, int64_t nbytes,
                                                  AbsDesc* __restrict__ A, int na, uint64_t* __restrict__ k1,
                                                  uint64_t* __restrict__ k2, unsigned long long* __restrict__ nent) {
  __shared__ int64_t sW[4];
  __shared__ unsigned long long sBase;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * SS_BYTES;
  int64_t cnt = 0;
  int a;
  for (int q = 0; q < SS_BYTES; q++)
    if (b0 + q < nbytes) cnt += seg_urls(t, A, na, b0 + q, a);
  int64_t incl = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) sW[wv] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t tot = sW[0] + sW[1] + sW[2] + sW[3];
    sBase = tot > 0 ? atomicAdd(nent, (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  int64_t s0 = (int64_t)sBase + incl - cnt;
  for (int w = 0; w < wv; w++) s0 += sW[w];
  if (cnt == 0) return;
  for (int q = 0; q < SS_BYTES; q++) {
    const int64_t b = b0 + q;
    if (b >= nbytes) break;
    const int64_t c = seg_urls(t, A, na, b, a);
    if (c == 0) continue;
    uint64_t hostpart = 0;  // url chars 6..11 = the host
    for (int j = 0; j < 6; j++) hostpart = (hostpart << 6) | (uint64_t)acode(t[b + j]);
    const uint32_t w = (uint32_t)A[a].word;
    for (int64_t k = 0; k < c; k++) {
      uint64_t x = 0;
      for (int j = 0; j < 6; j++) x = (x << 6) | (uint64_t)acode(t[b + 7 + 6 * k + j]);
      // 72-bit key: chars 0..5 (36 bits), host (36 bits); hi = top 64, lo = low 8
      k1[s0 + k] = (x << 28) | (hostpart >> 8);
      k2[s0 + k] = ((hostpart & 0xFF) << 40) | ((uint64_t)w << 32) | (uint64_t)(uint32_t)a;
    }
    s0 += c;
  }
}

__global__ void k_iota(uint32_t* __restrict__ v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}
__global__ void k_gather_key(const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t n,
                             uint64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

__device__ __forceinline__ bool same_url(const uint64_t* k1, const uint64_t* k2, int64_t i, int64_t j) {
  return k1[i] == k1[j] && (k2[i] >> 40) == (k2[j] >> 40);
}

// per (url, word): the newest abstract's peer (addAbstract keeps the replacing set);
// per word: distinct urls (the map sizes joinConstructive orders by)
__global__ void k_ss_count(const uint64_t* __restrict__ k1, const uint64_t* __restrict__ k2, int64_t n,
                           int32_t* __restrict__ wcount, uint32_t* __restrict__ head) {
  __shared__ int32_t sW[32];
  if (threadIdx.x < 32) sW[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint32_t w = (uint32_t)(k2[i] >> 32) & 0xFF;
    const bool last_w = i == n - 1 || !same_url(k1, k2, i, i + 1) || ((uint32_t)(k2[i + 1] >> 32) & 0xFF) != w;
    if (last_w) atomicAdd(&sW[w], 1);
    head[i] = (i == 0 || !same_url(k1, k2, i, i - 1)) ? 1u : 0u;
  }
  __syncthreads();
  if (threadIdx.x < 32 && sW[threadIdx.x]) atomicAdd(&wcount[threadIdx.x], sW[threadIdx.x]);
}

// one thread per url: joined? -> the first join word's peer; words of that peer
__global__ void k_ss_join(const uint64_t* __restrict__ k1, const uint64_t* __restrict__ k2, int64_t n,
                          const uint32_t* __restrict__ head, const AbsDesc* __restrict__ A, uint32_t jmask,
                          int32_t w0, int32_t* __restrict__ jpeer, uint32_t* __restrict__ pmask) {
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= n) return;
  jpeer[h] = -1;
  if (!head[h]) return;
  int32_t peer_w[32];
  uint32_t mask = 0;
  for (int64_t i = h; i < n && (i == h || !head[i]); i++) {
    const uint32_t w = (uint32_t)(k2[i] >> 32) & 0xFF;
    peer_w[w] = A[(uint32_t)k2[i]].peer;  // ascending abstract index: the last one stays
    mask |= 1u << w;
  }
  if ((mask & jmask) != jmask) return;
  const int32_t p0 = peer_w[w0];
  jpeer[h] = p0;
  uint32_t pw = 0;
  for (int w = 0; w < 32; w++)
    if ((mask >> w) & 1u && peer_w[w] == p0) pw |= 1u << w;
  // most threads of a wave share the few words masks of a peer: skip repeated global atomics
  if ((__ldg(&pmask[p0]) & pw) != pw) atomicOr(&pmask[p0], pw);
}

__global__ void k_ss_flags(const int32_t* __restrict__ jpeer, int64_t n, uint32_t* __restrict__ f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = jpeer[i] >= 0 ? 1u : 0u;
}

// joined urls in url order (incl = inclusive scan of the flags)
__global__ void k_ss_compact(const uint64_t* __restrict__ k1, const uint64_t* __restrict__ k2,
                             const int32_t* __restrict__ jpeer, const uint32_t* __restrict__ incl, int64_t n,
                             uint8_t* __restrict__ urls, uint32_t* __restrict__ peers, uint32_t* __restrict__ order) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || jpeer[i] < 0) return;
  const int64_t o = (int64_t)incl[i] - 1;
  const uint64_t hi = k1[i], lo = (k2[i] >> 40) & 0xFF;
  uint8_t* u = urls + o * 12;
  for (int j = 0; j < 10; j++) u[j] = achar((int)((hi >> (58 - 6 * j)) & 63));
  const int c10 = (int)(((hi & 0xF) << 2) | (lo >> 6));
  u[10] = achar(c10);
  u[11] = achar((int)(lo & 63));
  peers[o] = (uint32_t)jpeer[i];
  order[o] = (uint32_t)o;
}

__global__ void k_ss_gather_urls(const uint8_t* __restrict__ src, const uint32_t* __restrict__ idx, int64_t n,
                                 uint8_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int j = 0; j < 12; j++) dst[i * 12 + j] = src[(int64_t)idx[i] * 12 + j];
}

int ceil_bits(uint64_t x) {
  int b = 1;
  while (b < 64 && (1ull << b) <= x) b++;
  return b;
}

}  // namespace

extern "C" int yrwi_index_abstracts(yrwi_ctx* ctx, const uint8_t* terms, int32_t nterms, const uint8_t* exclude_term,
                                    char* out, int64_t cap, int64_t* offsets, int32_t* nout) {
  if (!ctx || nterms < 0 || (nterms > 0 && (!terms || !offsets)) || cap < 0 || (cap > 0 && !out) || !nout)
    return YRWI_E_ARG;
  *nout = 0;
  for (int32_t i = 0; i <= nterms; i++) offsets[i] = 0;
  hipSetDevice(ctx->device);
  drain(ctx);
  // AbstractIndex.searchConjunction (:96-128): every term needs a non-empty container
  std::vector<const ListRec*> ls;
  for (int32_t i = 0; i < nterms; i++) {
    KeyT k;
    if (!key_of(terms + 12 * i, &k)) return ctx->fail(YRWI_E_HASH, "term hash not well-formed");
    auto it = ctx->lists.find(k);
    if (it == ctx->lists.end() || it->second.n == 0) return 0;
    ls.push_back(&it->second);
  }
  const ListRec* ex = nullptr;
  if (exclude_term) {
    KeyT k;
    if (!key_of(exclude_term, &k)) return ctx->fail(YRWI_E_HASH, "exclude term hash not well-formed");
    auto it = ctx->lists.find(k);
    if (it != ctx->lists.end() && it->second.n > 0) ex = &it->second;
  }
  Lane* L = ctx->lanes[0];
  hipStream_t st = L->stream;
  int64_t pos = 0;
  for (int32_t t = 0; t < nterms; t++) {
    if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
    const ListRec& R = *ls[(size_t)t];
    const int64_t n = R.n;
    const int ni = (int)n;
    uint64_t* keys = arena_alloc<uint64_t>(L, n);
    uint64_t* keys2 = arena_alloc<uint64_t>(L, n);
    uint32_t* vals = arena_alloc<uint32_t>(L, n);
    uint32_t* vals2 = arena_alloc<uint32_t>(L, n);
    uint32_t* flag = arena_alloc<uint32_t>(L, n);
    uint32_t* g1 = arena_alloc<uint32_t>(L, n);
    unsigned long long* d_nex = arena_alloc<unsigned long long>(L, 1);
    uint8_t* d_out = arena_alloc<uint8_t>(L, 14 * n + 2);
    if (!keys || !keys2 || !vals || !vals2 || !flag || !g1 || !d_nex || !d_out) return ctx->fail(YRWI_E_NOMEM, "arena");
    size_t t1 = 0, t2 = 0;
    HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t1, keys, keys2, vals, vals2, ni, 0, 49, st));
    HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(nullptr, t2, flag, g1, ni, st));
    void* tmp = arena_alloc<uint8_t>(L, (int64_t)std::max(t1, t2));
    if (!tmp) return ctx->fail(YRWI_E_NOMEM, "arena");
    HIPCHK(ctx, hipMemsetAsync(d_nex, 0, 8, st));
    hipLaunchKernelGGL(k_ca_keys, dim3(nb(n)), dim3(256), 0, st, R.rows, R.khi, R.klo, n, ex ? ex->khi : nullptr,
                       ex ? ex->klo : nullptr, ex ? ex->n : (int64_t)0, keys, vals, d_nex);
    HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t1, keys, keys2, vals, vals2, ni, 0, 49, st));
    hipLaunchKernelGGL(k_ca_heads, dim3(nb(n)), dim3(256), 0, st, keys2, n, flag);
    HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(tmp, t2, flag, g1, ni, st));
    unsigned long long nex = 0;
    HIPCHK(ctx, hipMemcpyAsync(&nex, d_nex, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, lane_sync(L));
    const int64_t m = n - (int64_t)nex;  // postings left after the exclusion (sorted first)
    uint32_t G = 0;
    if (m > 0) {
      HIPCHK(ctx, hipMemcpyAsync(&G, g1 + (m - 1), 4, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, lane_sync(L));
    }
    const int64_t len = m > 0 ? 8 * (int64_t)G + 6 * m + 1 : 2;
    if (pos + len > cap) {
      offsets[t + 1] = pos + len;
      return ctx->fail(YRWI_E_ARG, "abstract output buffer too small");
    }
    if (m > 0) {
      hipLaunchKernelGGL(k_ca_write, dim3(nb(m)), dim3(256), 0, st, R.rows, keys2, vals2, g1, m, d_out);
      HIPCHK(ctx, hipGetLastError());
      HIPCHK(ctx, hipMemcpyAsync(out + pos, d_out, (size_t)len, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, lane_sync(L));
    } else {
      out[pos] = '{';
      out[pos + 1] = '}';
    }
    pos += len;
    offsets[t + 1] = pos;
  }
  *nout = nterms;
  return 0;
}

extern "C" int yrwi_secondary_search(yrwi_ctx* ctx, const yrwi_abstract* abs, int32_t nabs, int32_t nwords_query,
                                     const uint8_t mypeer[12], const uint8_t* checked, int32_t nchecked,
                                     uint8_t* join_urls, uint8_t* join_peers, int64_t cap, int64_t* njoin,
                                     yrwi_peer_request* plan, int32_t plan_cap, int32_t* nplan, uint8_t* plan_urls,
                                     uint8_t* words_out, int32_t* nwords) {
  if (!ctx || nabs < 0 || (nabs > 0 && !abs) || cap < 0 || !njoin || !nplan || !nwords || plan_cap < 0 ||
      (plan_cap > 0 && !plan) || nchecked < 0 || (nchecked > 0 && !checked) || !mypeer)
    return YRWI_E_ARG;
  *njoin = 0;
  *nplan = 0;
  *nwords = 0;
  // word and peer ranks in String order (the TreeMaps of the supervisor)
  auto less12 = [](const std::array<uint8_t, 12>& a, const std::array<uint8_t, 12>& b) {
    return std::memcmp(a.data(), b.data(), 12) < 0;
  };
  std::vector<std::array<uint8_t, 12>> words, peers;
  std::array<uint8_t, 12> x;
  int64_t nbytes = 0;
  for (int32_t i = 0; i < nabs; i++) {
    if (abs[i].len < 0 || (abs[i].len > 0 && !abs[i].text)) return ctx->fail(YRWI_E_ARG, "bad abstract");
    std::memcpy(x.data(), abs[i].word, 12);
    words.push_back(x);
    std::memcpy(x.data(), abs[i].peer, 12);
    peers.push_back(x);
    nbytes += abs[i].len;
  }
  std::sort(words.begin(), words.end(), less12);
  words.erase(std::unique(words.begin(), words.end()), words.end());
  std::sort(peers.begin(), peers.end(), less12);
  peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
  if (words.size() > 32) return ctx->fail(YRWI_E_ARG, "more than 32 words");
  *nwords = (int32_t)words.size();
  if (words_out)
    for (size_t i = 0; i < words.size(); i++) std::memcpy(words_out + 12 * i, words[i].data(), 12);
  // prepareSecondarySearch: only once every include word has its abstracts
  if (nabs == 0 || (int32_t)words.size() != nwords_query) return 0;
  auto rank_of = [&](const std::vector<std::array<uint8_t, 12>>& v, const uint8_t* h) {
    std::memcpy(x.data(), h, 12);
    return (int32_t)(std::lower_bound(v.begin(), v.end(), x, less12) - v.begin());
  };
  std::vector<AbsDesc> A((size_t)nabs);
  int64_t off = 0;
  for (int32_t i = 0; i < nabs; i++) {
    A[(size_t)i] = AbsDesc{off, abs[i].len, rank_of(words, abs[i].word), rank_of(peers, abs[i].peer), INT64_MAX, 0, 0};
    off += abs[i].len;
  }
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  hipStream_t st = L->stream;
  const int64_t maxent = nbytes / 6 + 1;
  uint8_t* d_text = arena_alloc<uint8_t>(L, nbytes);
  AbsDesc* d_abs = arena_alloc<AbsDesc>(L, nabs);
  unsigned long long* d_nent = arena_alloc<unsigned long long>(L, 1);
  uint64_t* k1 = arena_alloc<uint64_t>(L, maxent);
  uint64_t* k2 = arena_alloc<uint64_t>(L, maxent);
  if (!d_text || !d_abs || !d_nent || !k1 || !k2) return ctx->fail(YRWI_E_NOMEM, "arena");
  uint8_t* stg = stage_reserve(L, &L->out_stage, (size_t)std::max<int64_t>(nbytes, 4), true);
  if (!stg) return ctx->take(L, YRWI_E_HIP);
  for (int32_t i = 0; i < nabs; i++)
    if (abs[i].len) std::memcpy(stg + A[(size_t)i].off, abs[i].text, (size_t)abs[i].len);
  if (nbytes) HIPCHK(ctx, hipMemcpyAsync(d_text, stg, (size_t)nbytes, hipMemcpyHostToDevice, st));
  if (upload(L, d_abs, A)) return ctx->take(L, YRWI_E_HIP);
  HIPCHK(ctx, hipMemsetAsync(d_nent, 0, 8, st));
  if (nbytes) {
    hipLaunchKernelGGL(k_ss_bad, dim3(nb(nbytes)), dim3(256), 0, st, d_text, nbytes, d_abs, nabs);
    hipLaunchKernelGGL(k_ss_parse, dim3(nb((nbytes + SS_BYTES - 1) / SS_BYTES)), dim3(256), 0, st, d_text, nbytes, d_abs,
                       nabs, k1, k2, d_nent);
    HIPCHK(ctx, hipGetLastError());
  }
  unsigned long long nent = 0;
  HIPCHK(ctx, hipMemcpyAsync(&nent, d_nent, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(A.data(), d_abs, sizeof(AbsDesc) * (size_t)nabs, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, lane_sync(L));
  for (auto& D : A)
    if (D.err) return ctx->fail(YRWI_E_ARG, "malformed index abstract");
  const int64_t n = (int64_t)nent;
  // decompressIndex maps of the words (joinConstructive: an empty map -> empty join)
  std::vector<int32_t> wcount(words.size(), 0);
  uint64_t *k1b = nullptr, *k2b = nullptr;
  uint32_t* head = nullptr;
  if (n > 0) {
    const int ni = (int)n;
    uint64_t* k2a = arena_alloc<uint64_t>(L, n);
    uint64_t* k1a = arena_alloc<uint64_t>(L, n);
    k1b = arena_alloc<uint64_t>(L, n);
    k2b = arena_alloc<uint64_t>(L, n);
    uint32_t* v0 = arena_alloc<uint32_t>(L, n);
    uint32_t* v1 = arena_alloc<uint32_t>(L, n);
    uint32_t* v2 = arena_alloc<uint32_t>(L, n);
    head = arena_alloc<uint32_t>(L, n);
    int32_t* d_wc = arena_alloc<int32_t>(L, 32);
    if (!k2a || !k1a || !k1b || !k2b || !v0 || !v1 || !v2 || !head || !d_wc) return ctx->fail(YRWI_E_NOMEM, "arena");
    size_t t1 = 0, t2 = 0;
    const int b2 = 40 + 8;  // lo8 << 40 | word << 32 | abstract
    HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t1, k2, k2a, v0, v1, ni, 0, b2, st));
    HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t2, k1a, k1b, v0, v2, ni, 0, 64, st));
    void* tmp = arena_alloc<uint8_t>(L, (int64_t)std::max(t1, t2));
    if (!tmp) return ctx->fail(YRWI_E_NOMEM, "arena");
    hipLaunchKernelGGL(k_iota, dim3(nb(n)), dim3(256), 0, st, v0, n);
    HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t1, k2, k2a, v0, v1, ni, 0, b2, st));
    hipLaunchKernelGGL(k_gather_key, dim3(nb(n)), dim3(256), 0, st, k1, v1, n, k1a);
    hipLaunchKernelGGL(k_iota, dim3(nb(n)), dim3(256), 0, st, v0, n);
    HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t2, k1a, k1b, v0, v2, ni, 0, 64, st));
    hipLaunchKernelGGL(k_gather_key, dim3(nb(n)), dim3(256), 0, st, k2a, v2, n, k2b);
    HIPCHK(ctx, hipMemsetAsync(d_wc, 0, 32 * 4, st));
    hipLaunchKernelGGL(k_ss_count, dim3(nb(n)), dim3(256), 0, st, k1b, k2b, n, d_wc, head);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(wcount.data(), d_wc, 4 * words.size(), hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, lane_sync(L));
  }
  // joinConstructive order: Long.valueOf(size * 1000 + count) (an int), TreeMap put
  std::map<int32_t, int32_t> order;
  for (size_t w = 0; w < words.size(); w++) {
    if (wcount[w] == 0) return 0;
    order[(int32_t)((uint32_t)wcount[w] * 1000u + (uint32_t)w)] = (int32_t)w;
  }
  uint32_t jmask = 0;
  for (auto& kv : order) jmask |= 1u << kv.second;
  const int32_t w0 = order.begin()->second;
  int32_t* jpeer = arena_alloc<int32_t>(L, n);
  uint32_t* pmask = arena_alloc<uint32_t>(L, (int64_t)peers.size());
  uint32_t* f = arena_alloc<uint32_t>(L, n);
  uint32_t* incl = arena_alloc<uint32_t>(L, n);
  uint8_t* d_urls = arena_alloc<uint8_t>(L, 12 * n);
  uint8_t* d_urls2 = arena_alloc<uint8_t>(L, 12 * n);
  uint32_t* d_peer = arena_alloc<uint32_t>(L, n);
  uint32_t* d_peer2 = arena_alloc<uint32_t>(L, n);
  uint32_t* d_ord = arena_alloc<uint32_t>(L, n);
  uint32_t* d_ord2 = arena_alloc<uint32_t>(L, n);
  if (!jpeer || !pmask || !f || !incl || !d_urls || !d_urls2 || !d_peer || !d_peer2 || !d_ord || !d_ord2)
    return ctx->fail(YRWI_E_NOMEM, "arena");
  const int ni = (int)n;
  size_t t3 = 0, t4 = 0;
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(nullptr, t3, f, incl, ni, st));
  const int pbits = ceil_bits(peers.size());
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, t4, d_peer, d_peer2, d_ord, d_ord2, ni, 0, pbits, st));
  void* tmp2 = arena_alloc<uint8_t>(L, (int64_t)std::max(t3, t4));
  if (!tmp2) return ctx->fail(YRWI_E_NOMEM, "arena");
  HIPCHK(ctx, hipMemsetAsync(pmask, 0, 4 * peers.size(), st));
  hipLaunchKernelGGL(k_ss_join, dim3(nb(n)), dim3(256), 0, st, k1b, k2b, n, head, d_abs, jmask, w0, jpeer, pmask);
  hipLaunchKernelGGL(k_ss_flags, dim3(nb(n)), dim3(256), 0, st, jpeer, n, f);
  HIPCHK(ctx, hipcub::DeviceScan::InclusiveSum(tmp2, t3, f, incl, ni, st));
  hipLaunchKernelGGL(k_ss_compact, dim3(nb(n)), dim3(256), 0, st, k1b, k2b, jpeer, incl, n, d_urls, d_peer, d_ord);
  HIPCHK(ctx, hipGetLastError());
  uint32_t J = 0;
  HIPCHK(ctx, hipMemcpyAsync(&J, incl + (n - 1), 4, hipMemcpyDeviceToHost, st));
  std::vector<uint32_t> pm(peers.size());
  HIPCHK(ctx, hipMemcpyAsync(pm.data(), pmask, 4 * peers.size(), hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, lane_sync(L));
  *njoin = J;
  if ((int64_t)J > cap) return ctx->fail(YRWI_E_ARG, "join output buffer too small");
  if (J == 0) return 0;
  // urls grouped by peer (stable: url order inside a peer)
  HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp2, t4, d_peer, d_peer2, d_ord, d_ord2, (int)J, 0, pbits, st));
  hipLaunchKernelGGL(k_ss_gather_urls, dim3(nb(J)), dim3(256), 0, st, d_urls, d_ord2, (int64_t)J, d_urls2);
  HIPCHK(ctx, hipGetLastError());
  std::vector<uint32_t> jp(J), gp(J);
  std::vector<uint8_t> gu((size_t)J * 12);
  if (join_urls) HIPCHK(ctx, hipMemcpyAsync(join_urls, d_urls, (size_t)J * 12, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(jp.data(), d_peer, 4 * (size_t)J, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(gp.data(), d_peer2, 4 * (size_t)J, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(gu.data(), d_urls2, (size_t)J * 12, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, lane_sync(L));
  if (join_peers)
    for (uint32_t i = 0; i < J; i++) std::memcpy(join_peers + 12 * (size_t)i, peers[jp[i]].data(), 12);
  // the requests: peers in String order, minus ourselves and the peers already asked
  std::vector<std::array<uint8_t, 12>> chk;
  for (int32_t i = 0; i < nchecked; i++) {
    std::memcpy(x.data(), checked + 12 * i, 12);
    chk.push_back(x);
  }
  int32_t np = 0;
  int64_t uoff = 0;
  for (uint32_t i = 0; i < J;) {
    uint32_t e = i;
    while (e < J && gp[e] == gp[i]) e++;
    const auto& ph = peers[gp[i]];
    const bool skip = std::memcmp(ph.data(), mypeer, 12) == 0 ||
                      std::find(chk.begin(), chk.end(), ph) != chk.end() || pm[gp[i]] == 0;
    if (!skip) {
      if (np >= plan_cap) return ctx->fail(YRWI_E_ARG, "plan buffer too small");
      yrwi_peer_request& R = plan[np++];
      std::memcpy(R.peer, ph.data(), 12);
      R.words = pm[gp[i]];
      R.url_off = uoff;
      R.url_n = (int64_t)(e - i);
      if (plan_urls) std::memcpy(plan_urls + 12 * uoff, gu.data() + 12 * (size_t)i, 12 * (size_t)(e - i));
      uoff += e - i;
    }
    i = e;
  }
  *nplan = np;
  return 0;
}
