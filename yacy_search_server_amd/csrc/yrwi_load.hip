// yrwi_load.hip -- YaCy BLOB heap files -> HBM-resident posting lists
// (SURVEY.md §8f row 1).  Paths relative to /root/reference/source/net/yacy.
//
// A heap file is a sequence of records [int32 BE reclen][12-byte term hash]
// [exported RowSet] (kelondro/blob/HeapWriter.java:57-63,114-124); the export
// is a 14-byte header (size-4, lastread-2, lastwrote-2, orderkey-2,
// orderbound-4) followed by size 40-byte WordReferenceRows
// (kelondro/index/RowCollection.java:175-231).  The loader restates
//   * the heap scan of HeapReader.initIndexReadFromHeap (:250-304): reclen 0
//     ends the file, key[0] == 0 is a free record, keys that are not
//     well-formed Base64 are skipped, a key seen again replaces the earlier one;
//   * RowSet.importRowSet (RowSet.java:81-109): size < 0 or orderbound < 0 is an
//     empty set, size*40 != len-14 is a SpaceExceededException, which drops the
//     term's whole BLOB part (IndexCell.get :357-360);
//   * ArrayStack's file order (ArrayStack.java:182-229, oldest stamp first) and
//     ReferenceContainerArray.get's fold (:305-322) with RowSet.mergeEnum
//     (RowSet.java:506-559): on equal url hashes the older file's row wins;
//   * IndexCell.get (:353-386): the lists already in the context play the RAM
//     cache, merged below the files (the file row wins).
// Rows past orderbound (never written by exportCollection, which sorts first)
// are sorted stably on the host and the first of equal url hashes is kept.
//
// Device side: file rows are uploaded through pinned staging into HBM,
// validated and keyed by k_validate, and multi-source terms are merged on the
// GPU by rank (k_union_*): every row's output slot is its index plus its rank
// in the other list, minus the duplicates ahead of it.

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hipcub/hipcub.hpp>

#include "yrwi_host.h"

using namespace yrwi;

namespace {

__device__ __forceinline__ int64_t lb_key(const uint64_t* __restrict__ kh, const uint8_t* __restrict__ kl, int64_t n,
                                          uint64_t h, uint32_t l) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const uint64_t mh = kh[mid];
    if (mh < h || (mh == h && (uint32_t)kl[mid] < l)) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void copy_row(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src) {
  const uint64_t* s = reinterpret_cast<const uint64_t*>(src);  // rows are 8-byte aligned (40 B, 256 B bases)
  uint64_t* d = reinterpret_cast<uint64_t*>(dst);
#pragma unroll
  for (int i = 0; i < 5; i++) d[i] = s[i];
}

// B rows: slot in A (lower bound) and whether B's key is absent from A (kept)
__global__ void k_union_b(DList A, DList B, int64_t* __restrict__ lbA, int32_t* __restrict__ keep) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B.n) return;
  const uint64_t h = B.khi[j];
  const uint32_t l = B.klo[j];
  const int64_t p = lb_key(A.khi, A.klo, A.n, h, l);
  lbA[j] = p;
  keep[j] = (p < A.n && A.khi[p] == h && (uint32_t)A.klo[p] == l) ? 0 : 1;
}

// A rows go to i + (kept B rows before A[i]); rB = exclusive scan of keep (nB + 1 entries)
__global__ void k_union_a(DList A, DList B, const int64_t* __restrict__ rB, uint64_t* __restrict__ okh,
                          uint8_t* __restrict__ okl, uint8_t* __restrict__ orows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  const uint64_t h = A.khi[i];
  const uint32_t l = A.klo[i];
  const int64_t pos = i + rB[lb_key(B.khi, B.klo, B.n, h, l)];
  okh[pos] = h;
  okl[pos] = (uint8_t)l;
  copy_row(orows + pos * YRWI_ROW_BYTES, A.rows + i * YRWI_ROW_BYTES);
}

__global__ void k_union_bs(DList B, const int64_t* __restrict__ lbA, const int32_t* __restrict__ keep,
                           const int64_t* __restrict__ rB, uint64_t* __restrict__ okh, uint8_t* __restrict__ okl,
                           uint8_t* __restrict__ orows) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B.n || !keep[j]) return;
  const int64_t pos = rB[j] + lbA[j];
  okh[pos] = B.khi[j];
  okl[pos] = B.klo[j];
  copy_row(orows + pos * YRWI_ROW_BYTES, B.rows + j * YRWI_ROW_BYTES);
}

unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

// ---------------------------------------------------------------- host side
inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

struct Seg {
  const uint8_t* blob;  // exported RowSet
  int64_t len;
};

struct MappedFile {
  const uint8_t* p = nullptr;
  size_t n = 0;
  ~MappedFile() {
    if (p && n) munmap(const_cast<uint8_t*>(p), n);
  }
};

bool wellformed(const uint8_t* k) {
  for (int i = 0; i < 12; i++)
    if (AHP[k[i]] < 0) return false;
  return true;
}

// stamp "<prefix>.<17 digits>.blob" (ArrayStack.java:187-190); empty if absent
std::string stamp_of(const std::string& path) {
  const std::string suf = ".blob";
  if (path.size() < 23 || path.compare(path.size() - suf.size(), suf.size(), suf) != 0) return "";
  const size_t e = path.size() - suf.size();
  if (path[e - 18] != '.') return "";
  for (size_t i = e - 17; i < e; i++)
    if (path[i] < '0' || path[i] > '9') return "";
  return path.substr(e - 17, 17);
}

// A device list being assembled (arena or index memory).
struct DevList {
  uint64_t* khi = nullptr;
  uint8_t* klo = nullptr;
  uint8_t* rows = nullptr;
  int64_t n = 0;
  DList dl() const { return DList{khi, klo, rows, n, nullptr}; }
};

}  // namespace

// Upload n host rows into fresh device arrays (from `mem`) and key/validate them.
static int upload_rows(yrwi_ctx* ctx, Lane* L, Arena* mem, const uint8_t* rows, int64_t n, DevList* out,
                       int32_t* herr) {
  out->n = n;
  out->rows = mem->alloc((size_t)n * 40);
  out->khi = reinterpret_cast<uint64_t*>(mem->alloc((size_t)n * 8));
  out->klo = mem->alloc((size_t)n);
  int32_t* derr = reinterpret_cast<int32_t*>(L->arena.alloc(4));
  if (!out->rows || !out->khi || !out->klo || !derr) return ctx->fail(YRWI_E_NOMEM, "device allocation (load)");
  // pinned staging in 16 MiB pieces (pageable copies are staged by the runtime anyway)
  const size_t piece = (size_t)16 << 20, total = (size_t)n * 40;
  uint8_t* stg = stage_reserve(L, &L->stage, 2 * piece, true);
  if (!stg) return ctx->take(L, YRWI_E_HIP);
  hipEvent_t done[2] = {L->event(), L->event()};
  bool used[2] = {false, false};
  for (size_t off = 0, k = 0; off < total; off += piece, k ^= 1) {
    const size_t m = std::min(piece, total - off);
    if (used[k]) HIPCHK(ctx, hipEventSynchronize(done[k]));
    std::memcpy(stg + k * piece, rows + off, m);
    HIPCHK(ctx, hipMemcpyAsync(out->rows + off, stg + k * piece, m, hipMemcpyHostToDevice, L->stream));
    HIPCHK(ctx, hipEventRecord(done[k], L->stream));
    used[k] = true;
  }
  HIPCHK(ctx, hipMemsetAsync(derr, 0, 4, L->stream));
  if (launch_validate_rows(out->rows, n, out->khi, out->klo, derr, L->stream)) return ctx->fail(YRWI_E_HIP, "validate");
  HIPCHK(ctx, hipMemcpyAsync(herr, derr, 4, hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, lane_sync(L));
  return 0;
}

// RowSet.mergeEnum(A, B) on the device: A's row wins on equal url hashes.
static int union_lists(yrwi_ctx* ctx, Lane* L, Arena* mem, const DList& A, const DList& B, DevList* out) {
  if (B.n == 0 || A.n == 0) {
    const DList& S = A.n ? A : B;
    out->n = S.n;
    out->khi = const_cast<uint64_t*>(S.khi);
    out->klo = const_cast<uint8_t*>(S.klo);
    out->rows = const_cast<uint8_t*>(S.rows);
    return 0;
  }
  int64_t* lbA = arena_alloc<int64_t>(L, B.n);
  int32_t* keep = arena_alloc<int32_t>(L, B.n + 1);
  int64_t* rB = arena_alloc<int64_t>(L, B.n + 1);
  if (!lbA || !keep || !rB) return ctx->fail(YRWI_E_NOMEM, "device allocation (union)");
  HIPCHK(ctx, hipMemsetAsync(keep + B.n, 0, 4, L->stream));
  hipLaunchKernelGGL(k_union_b, dim3(blocks(B.n)), dim3(256), 0, L->stream, A, B, lbA, keep);
  size_t tmp = 0;
  HIPCHK(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, keep, rB, (int)(B.n + 1), L->stream));
  void* dtmp = L->arena.alloc(tmp);
  if (!dtmp) return ctx->fail(YRWI_E_NOMEM, "device allocation (scan)");
  HIPCHK(ctx, hipcub::DeviceScan::ExclusiveSum(dtmp, tmp, keep, rB, (int)(B.n + 1), L->stream));
  int64_t kept = 0;
  HIPCHK(ctx, hipMemcpyAsync(&kept, rB + B.n, 8, hipMemcpyDeviceToHost, L->stream));
  HIPCHK(ctx, lane_sync(L));
  out->n = A.n + kept;
  out->rows = mem->alloc((size_t)out->n * 40);
  out->khi = reinterpret_cast<uint64_t*>(mem->alloc((size_t)out->n * 8));
  out->klo = mem->alloc((size_t)out->n);
  if (!out->rows || !out->khi || !out->klo) return ctx->fail(YRWI_E_NOMEM, "device allocation (union)");
  hipLaunchKernelGGL(k_union_a, dim3(blocks(A.n)), dim3(256), 0, L->stream, A, B, rB, out->khi, out->klo, out->rows);
  hipLaunchKernelGGL(k_union_bs, dim3(blocks(B.n)), dim3(256), 0, L->stream, B, lbA, keep, rB, out->khi, out->klo,
                     out->rows);
  HIPCHK(ctx, hipGetLastError());
  return 0;
}

// rows of this context's url-hash shard: first character c with c >> (6 - log2 W) == rank
// (Distribution.verticalDHTPosition, Distribution.java:153-158); rows are sorted by key
static void shard_range(const yrwi_ctx* ctx, const uint8_t* rows, int64_t n, int64_t* lo, int64_t* hi) {
  *lo = 0;
  *hi = n;
  if (ctx->world <= 1) return;
  int bits = 0;
  while ((1 << bits) < ctx->world) bits++;
  auto part = [&](int64_t i) { return AHP[rows[i * 40]] >> (6 - bits); };
  int64_t a = 0, b = n;
  while (a < b) {
    int64_t m = (a + b) / 2;
    if (part(m) < ctx->rank) a = m + 1; else b = m;
  }
  *lo = a;
  b = n;
  while (a < b) {
    int64_t m = (a + b) / 2;
    if (part(m) <= ctx->rank) a = m + 1; else b = m;
  }
  *hi = a;
}

extern "C" int yrwi_load_heaps(yrwi_ctx* ctx, const char* const* paths, int32_t npaths, int32_t flags,
                               yrwi_load_stats* st) {
  if (!ctx || npaths < 0 || (npaths > 0 && !paths)) return YRWI_E_ARG;
  yrwi_load_stats S;
  std::memset(&S, 0, sizeof(S));
  hipSetDevice(ctx->device);
  drain(ctx);
  Lane* L = ctx->lanes[0];
  // ---- file order
  std::vector<std::string> files;
  if (flags & YRWI_LOAD_ORDER_BY_NAME) {
    std::vector<std::pair<std::string, std::string>> st2;
    for (int i = 0; i < npaths; i++) {
      std::string p = paths[i] ? paths[i] : "", s = stamp_of(p);
      if (!s.empty()) st2.push_back({s, p});
    }
    std::stable_sort(st2.begin(), st2.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (auto& x : st2) files.push_back(x.second);
  } else {
    for (int i = 0; i < npaths; i++) files.push_back(paths[i] ? paths[i] : "");
  }
  // ---- scan every heap (HeapReader.initIndexReadFromHeap :250-304)
  std::vector<MappedFile> maps(files.size());
  std::map<KeyT, std::vector<std::pair<int, Seg>>> terms;  // term -> (file, blob) in file order
  for (size_t f = 0; f < files.size(); f++) {
    const int fd = open(files[f].c_str(), O_RDONLY);
    if (fd < 0) return ctx->fail(YRWI_E_ARG, "cannot open " + files[f]);
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
      close(fd);
      return ctx->fail(YRWI_E_ARG, "cannot stat " + files[f]);
    }
    const size_t len = (size_t)sb.st_size;
    if (len > 0) {
      void* p = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) {
        close(fd);
        return ctx->fail(YRWI_E_ARG, "cannot map " + files[f]);
      }
      madvise(p, len, MADV_SEQUENTIAL);
      maps[f].p = static_cast<const uint8_t*>(p);
      maps[f].n = len;
    }
    close(fd);
    S.files++;
    std::unordered_map<KeyT, Seg, KeyHash> recs;
    size_t seek = 0;
    const uint8_t* d = maps[f].p;
    while (seek + 4 + 12 <= len) {
      const int32_t reclen = (int32_t)be32(d + seek);
      if (reclen == 0) break;  // "very bad file inconsistency": the rest is cut off
      const uint8_t* key = d + seek + 4;
      if (key[0] == 0) {
        S.free_records++;
      } else if (!wellformed(key)) {
        S.bad_keys++;
      } else if (reclen >= 12 && seek + 4 + (size_t)reclen <= len) {
        KeyT k;
        key_of(key, &k);
        recs[k] = Seg{key + 12, (int64_t)reclen - 12};  // a key seen again replaces the earlier record
        S.records++;
      }
      if (reclen < 0) break;
      seek += 4 + (size_t)reclen;
    }
    for (auto& r : recs) terms[r.first].push_back({(int)f, r.second});
  }
  // ---- per term: import, fold the files (oldest first), merge the RAM part below
  std::vector<uint8_t> sorted_tmp;
  for (auto& T : terms) {
    if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
    bool poisoned = false;
    struct Src {
      const uint8_t* rows;
      int64_t n;
      std::vector<uint8_t> own;
    };
    std::vector<Src> srcs;
    for (auto& fs : T.second) {
      const Seg& g = fs.second;
      if (g.len < 14) continue;  // importRowSet: empty set
      const int32_t size = (int32_t)be32(g.blob), ob = (int32_t)be32(g.blob + 10);
      if (size < 0 || ob < 0) continue;
      if ((int64_t)size * 40 != g.len - 14) {
        poisoned = true;  // SpaceExceededException: IndexCell.get drops the BLOB part
        break;
      }
      Src s{g.blob + 14, size, {}};
      if (ob < size) {  // unsorted tail: stable sort, first of equal url hashes kept
        std::vector<std::pair<KeyT, int64_t>> ks((size_t)size);
        for (int64_t i = 0; i < size; i++) {
          if (!key_of(s.rows + i * 40, &ks[(size_t)i].first)) { poisoned = true; break; }
          ks[(size_t)i].second = i;
        }
        if (poisoned) break;
        std::stable_sort(ks.begin(), ks.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
        for (size_t i = 0; i < ks.size(); i++) {
          if (i > 0 && ks[i].first == ks[i - 1].first) continue;
          s.own.insert(s.own.end(), s.rows + ks[i].second * 40, s.rows + ks[i].second * 40 + 40);
        }
        s.rows = s.own.data();
        s.n = (int64_t)(s.own.size() / 40);
      }
      int64_t lo, hi;
      shard_range(ctx, s.rows, s.n, &lo, &hi);
      s.rows += lo * 40;
      s.n = hi - lo;
      if (s.n > 0) srcs.push_back(std::move(s));
    }
    if (poisoned) {
      S.dropped_terms++;
      srcs.clear();
    }
    auto it = ctx->lists.find(T.first);
    const bool has_ram = it != ctx->lists.end() && it->second.n > 0;
    if (srcs.empty()) continue;  // nothing from the files: the RAM list stays as it is
    // fold in HBM; intermediate lists in the lane arena, the final one in index memory
    DevList acc;
    bool failed = false;
    for (size_t i = 0; i < srcs.size() && !failed; i++) {
      const bool last = i + 1 == srcs.size() && !has_ram;
      DevList cur;
      int32_t herr = 0;
      Arena* mem = (srcs.size() == 1 && !has_ram) ? &ctx->index_mem : &L->arena;
      if (int rc = upload_rows(ctx, L, mem, srcs[i].rows, srcs[i].n, &cur, &herr)) return rc;
      if (herr) {
        failed = true;  // malformed url hash, empty language cell or unsorted rows
        break;
      }
      if (i == 0) {
        acc = cur;
      } else {
        DevList u;
        if (int rc = union_lists(ctx, L, last ? &ctx->index_mem : &L->arena, acc.dl(), cur.dl(), &u)) return rc;
        acc = u;
      }
    }
    if (failed) {
      S.dropped_terms++;
      continue;
    }
    if (has_ram) {
      DevList u;
      if (int rc = union_lists(ctx, L, &ctx->index_mem, acc.dl(), it->second.dl(), &u)) return rc;
      acc = u;
    }
    HIPCHK(ctx, lane_sync(L));
    if (acc.n > MAX_LIST) {
      S.dropped_terms++;
      continue;
    }
    ListRec R;
    R.khi = acc.khi;
    R.klo = acc.klo;
    R.rows = acc.rows;
    R.n = acc.n;
    const int64_t old_n = has_ram ? it->second.n : 0;
    ctx->npostings -= old_n;
    ctx->lists[T.first] = R;
    ctx->npostings += R.n;
    index_changed(ctx, T.first, old_n, true);
    S.terms++;
    S.postings += R.n;
  }
  if (begin_pass(L)) return ctx->take(L, YRWI_E_HIP);
  if (st) *st = S;
  return 0;
}
