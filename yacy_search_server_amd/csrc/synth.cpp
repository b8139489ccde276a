// synth.cpp -- deterministic synthetic RWI generator (host C++, multithreaded).
//
// Produces posting lists in exactly the reference's on-heap layout: per term a
// sorted run of 40-byte WordReferenceRow rows (WordReferenceRow.java:49-72,
// RowSet chunkcache order RowSet.java:419-423).  The distributions follow
// SURVEY.md §8(d):
//   * URL universe U split into 64 chunks by the first url-hash character
//     (YaCy's vertical DHT partition, Distribution.java:153-158), so that a
//     GPU shard can generate only the chunks it owns;
//   * url hash chars 0-5 uniform, chars 6-11 = host hash (5 chars) + host flag
//     char alpha[(https?32:0)|(tld<<2)|domlenKey] (DigestURL.java:271-289);
//     hosts drawn Zipf(s_host) from a pool;
//   * per-term document frequency df ~ Zipf(s_df) over the vocabulary, clipped
//     below the reference's 53,687,091-row container limit (RowSet.java:90-92);
//     each term's list is a Bernoulli(df/U) subset of the URL universe;
//   * feature bytes drawn as the indexer stores them (Segment.java:716-730);
//     stored worddistance is always 0 (WordReferenceRow.java:198).
// Every (term, chunk) pair has its own splitmix64 stream, so the output does
// not depend on thread count or on which chunks are generated.

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

const char* ALPHA = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
inline uint64_t hash3(uint64_t a, uint64_t b, uint64_t c) { return mix64(mix64(mix64(a) ^ b) ^ c); }

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    s += 0x9E3779B97F4A7C15ULL;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  double u01() { return ((next() >> 11) + 0.5) * (1.0 / 9007199254740992.0); }  // (0,1)
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

enum : uint64_t { TAG_HOST = 1, TAG_DOC = 2, TAG_WORD = 3, TAG_LIST = 4, TAG_TERM = 5, TAG_HH = 6, TAG_Q = 7 };

}  // namespace

extern "C" {

typedef struct yrwi_synth_cfg {
  uint64_t seed;
  int64_t n_urls;      // U, rounded down to a multiple of 64 internally
  int32_t n_terms;     // V
  int32_t n_hosts;     // host pool size
  int64_t n_postings;  // target P (sum of df before clipping)
  double zipf_df;      // exponent of df over term rank (0.8)
  double zipf_host;    // exponent of host popularity (1.1)
  int64_t df_clip;     // max df (<= 53,687,091)
  int32_t chunk_lo;    // generate only url chunks [chunk_lo, chunk_hi) of 64
  int32_t chunk_hi;
} yrwi_synth_cfg;

void yrwi_synth_default(yrwi_synth_cfg* c) {
  c->seed = 0x5941437900000001ULL;
  c->n_urls = 1000000;
  c->n_terms = 10000;
  c->n_hosts = 50000;
  c->n_postings = 10000000;
  c->zipf_df = 0.8;
  c->zipf_host = 1.1;
  c->df_clip = 50000000;
  c->chunk_lo = 0;
  c->chunk_hi = 64;
}

// df of every term (term id = rank, 0 = most frequent).
void yrwi_synth_df(const yrwi_synth_cfg* c, int64_t* df) {
  double h = 0;
  for (int32_t r = 1; r <= c->n_terms; r++) h += std::pow((double)r, -c->zipf_df);
  for (int32_t r = 1; r <= c->n_terms; r++) {
    double v = (double)c->n_postings * std::pow((double)r, -c->zipf_df) / h;
    int64_t d = (int64_t)std::llround(v);
    if (d < 1) d = 1;
    d = std::min<int64_t>(d, c->df_clip);
    d = std::min<int64_t>(d, c->n_urls);
    df[r - 1] = d;
  }
}

void yrwi_synth_term_hash(const yrwi_synth_cfg* c, int32_t t, uint8_t out[12]) {
  uint64_t x = hash3(c->seed, TAG_TERM, (uint64_t)t);
  uint64_t y = hash3(c->seed ^ 0xA5A5A5A5ULL, TAG_TERM, (uint64_t)t);
  for (int j = 0; j < 10; j++) out[j] = (uint8_t)ALPHA[(x >> (6 * j)) & 63];
  out[10] = (uint8_t)ALPHA[y & 63];
  out[11] = (uint8_t)ALPHA[(y >> 6) & 63];
}

}  // extern "C"

namespace {

struct Gen {
  yrwi_synth_cfg c;
  int64_t Uc;            // urls per chunk
  unsigned __int128 stride;  // key stride inside a chunk (2^66 / Uc)
  uint64_t rmod;         // number of free values above the 36 host bits
  std::vector<double> host_cdf;
  std::vector<int64_t> df;

  explicit Gen(const yrwi_synth_cfg* cfg) : c(*cfg) {
    Uc = std::max<int64_t>(1, c.n_urls / 64);
    stride = (((unsigned __int128)1) << 66) / (unsigned __int128)Uc;
    rmod = (uint64_t)(stride >> 36);
    if (rmod == 0) rmod = 1;
    host_cdf.resize((size_t)std::max(1, c.n_hosts));
    double acc = 0;
    for (int32_t k = 0; k < c.n_hosts; k++) {
      acc += std::pow((double)(k + 1), -c.zipf_host);
      host_cdf[(size_t)k] = acc;
    }
    for (auto& v : host_cdf) v /= acc;
    df.resize((size_t)c.n_terms);
    yrwi_synth_df(&c, df.data());
  }

  uint64_t host36(int64_t u) const {
    Rng r(hash3(c.seed, TAG_HOST, (uint64_t)u));
    double x = r.u01();
    size_t k = (size_t)(std::lower_bound(host_cdf.begin(), host_cdf.end(), x) - host_cdf.begin());
    if (k >= host_cdf.size()) k = host_cdf.size() - 1;
    uint64_t hh = hash3(c.seed, TAG_HH, (uint64_t)k);
    uint64_t h30 = hh & ((1ULL << 30) - 1);
    uint64_t https = (hh >> 30) & 1;
    uint64_t tld = (hh >> 31) & 7;
    uint64_t domlen = (hh >> 34) & 3;
    uint64_t flag = (https ? 32 : 0) | (tld << 2) | domlen;
    return (h30 << 6) | flag;
  }

  void url_hash(int64_t chunk, int64_t v, uint8_t* out) const {
    int64_t u = chunk * Uc + v;
    uint64_t rr = hash3(c.seed, TAG_DOC ^ 0x55, (uint64_t)u) % rmod;
    unsigned __int128 low = (unsigned __int128)v * stride + ((unsigned __int128)rr << 36) + host36(u);
    unsigned __int128 k72 = (((unsigned __int128)chunk) << 66) | low;
    for (int j = 0; j < 12; j++) out[j] = (uint8_t)ALPHA[(uint64_t)(k72 >> (6 * (11 - j))) & 63];
  }

  void row(int32_t t, int64_t chunk, int64_t v, uint8_t* r) const {
    int64_t u = chunk * Uc + v;
    std::memset(r, 0, 40);
    url_hash(chunk, v, r);
    Rng d(hash3(c.seed, TAG_DOC, (uint64_t)u));
    int a = 10957 + (int)d.below(20454 - 10957 + 1);
    int s = std::min(65535, a + 30 + (int)d.below(60));
    int ut = (int)d.below(21);
    double ln = std::exp(5.5 + 1.2 * std::sqrt(-2.0 * std::log(d.u01())) * std::cos(6.283185307179586 * d.u01()));
    int w = (int)std::min(65535.0, std::max(1.0, ln));
    int p = std::max(1, w / 12);
    static const char* langs[6] = {"en", "de", "fr", "es", "it", "nl"};
    double lr = d.u01();
    int li = lr < 0.6 ? 0 : lr < 0.8 ? 1 : 2 + (int)d.below(4);
    auto geom = [&](Rng& g, double pz, int lo, int hi) {
      int v2 = lo;
      while (v2 < hi && g.u01() > pz) v2++;
      return v2;
    };
    int x = geom(d, 0.15, 0, 255);
    int y = geom(d, 0.08, 0, 255);
    int m = 16 + (int)d.below(240);
    int n = 1 + (int)d.below(15);
    uint32_t docflags = 0;
    if (d.u01() < 0.05) docflags |= 1u << 0;
    for (int b = 19; b <= 23; b++) if (d.u01() < 0.05) docflags |= 1u << b;
    Rng wd(hash3(c.seed ^ ((uint64_t)t << 20), TAG_WORD, (uint64_t)u));
    int hc = geom(wd, 0.45, 1, 255);
    int pos = 1 + (int)wd.below((uint64_t)std::min(w, 65535));
    int pip = 1 + (int)wd.below(40);
    int pop = 100 + (int)wd.below(156);
    uint32_t flags = docflags;
    static const double pbit[6] = {0.12, 0.2, 0.05, 0.1, 0.08, 0.15};
    for (int b = 24; b <= 29; b++) if (wd.u01() < pbit[b - 24]) flags |= 1u << b;
    r[12] = (uint8_t)(a >> 8); r[13] = (uint8_t)a;
    r[14] = (uint8_t)(s >> 8); r[15] = (uint8_t)s;
    r[16] = (uint8_t)ut;
    r[17] = (uint8_t)(w >> 8); r[18] = (uint8_t)w;
    r[19] = (uint8_t)(p >> 8); r[20] = (uint8_t)p;
    r[21] = 't';
    r[22] = (uint8_t)langs[li][0]; r[23] = (uint8_t)langs[li][1];
    r[24] = (uint8_t)x; r[25] = (uint8_t)y; r[26] = (uint8_t)m; r[27] = (uint8_t)n;
    r[28] = 0;
    // Bitfield byte order: bit b lives in byte b>>3, bit b%8 (Bitfield.java:88-93)
    r[29] = (uint8_t)(flags & 0xFF); r[30] = (uint8_t)((flags >> 8) & 0xFF);
    r[31] = (uint8_t)((flags >> 16) & 0xFF); r[32] = (uint8_t)((flags >> 24) & 0xFF);
    r[33] = (uint8_t)hc;
    r[34] = (uint8_t)(pos >> 8); r[35] = (uint8_t)pos;
    r[36] = (uint8_t)pip; r[37] = (uint8_t)pop;
    r[38] = 0;  // stored worddistance is always 0
    r[39] = 0;
  }

  // Bernoulli(df/U) selection inside one chunk via geometric skips.
  template <class F>
  int64_t walk(int32_t t, int64_t chunk, F&& emit) const {
    double q = (double)df[(size_t)t] / (double)(Uc * 64);
    int64_t n = 0;
    if (q >= 1.0) {
      for (int64_t v = 0; v < Uc; v++) { emit(v); n++; }
      return n;
    }
    Rng g(hash3(c.seed, TAG_LIST, ((uint64_t)t << 8) | (uint64_t)chunk));
    double lq = std::log1p(-q);
    int64_t v = -1;
    while (true) {
      double skip = std::floor(std::log(g.u01()) / lq);
      if (skip > (double)Uc) break;
      v += 1 + (int64_t)skip;
      if (v >= Uc) break;
      emit(v);
      n++;
    }
    return n;
  }
};

}  // namespace

extern "C" {

// Number of postings of every term (restricted to the configured chunks).
int yrwi_synth_counts(const yrwi_synth_cfg* cfg, int32_t nthreads, int64_t* counts) {
  Gen g(cfg);
  std::atomic<int32_t> next(0);
  auto work = [&]() {
    int32_t t;
    while ((t = next.fetch_add(1)) < g.c.n_terms) {
      int64_t n = 0;
      for (int64_t ch = g.c.chunk_lo; ch < g.c.chunk_hi; ch++) n += g.walk(t, ch, [](int64_t) {});
      counts[t] = n;
    }
  };
  std::vector<std::thread> th;
  for (int i = 0; i < std::max(1, nthreads); i++) th.emplace_back(work);
  for (auto& x : th) x.join();
  return 0;
}

// Fill the rows of terms [t0, t1) into `rows`; term t starts at row offsets[t]
// (offsets are relative to `rows`, as produced by an exclusive scan of counts).
int yrwi_synth_fill(const yrwi_synth_cfg* cfg, int32_t t0, int32_t t1, const int64_t* offsets,
                    uint8_t* rows, int32_t nthreads) {
  Gen g(cfg);
  std::atomic<int32_t> next(t0);
  auto work = [&]() {
    int32_t t;
    while ((t = next.fetch_add(1)) < t1) {
      uint8_t* out = rows + offsets[t - t0] * 40;
      for (int64_t ch = g.c.chunk_lo; ch < g.c.chunk_hi; ch++) {
        g.walk(t, ch, [&](int64_t v) {
          g.row(t, ch, v, out);
          out += 40;
        });
      }
    }
  };
  std::vector<std::thread> th;
  for (int i = 0; i < std::max(1, nthreads); i++) th.emplace_back(work);
  for (auto& x : th) x.join();
  return 0;
}

// Fill the rows of an arbitrary term subset: term terms[i] starts at row offsets[i].
int yrwi_synth_fill_terms(const yrwi_synth_cfg* cfg, const int32_t* terms, int32_t nterms, const int64_t* offsets,
                          uint8_t* rows, int32_t nthreads) {
  Gen g(cfg);
  std::atomic<int32_t> next(0);
  auto work = [&]() {
    int32_t i;
    while ((i = next.fetch_add(1)) < nterms) {
      const int32_t t = terms[i];
      uint8_t* out = rows + offsets[i] * 40;
      for (int64_t ch = g.c.chunk_lo; ch < g.c.chunk_hi; ch++) {
        g.walk(t, ch, [&](int64_t v) {
          g.row(t, ch, v, out);
          out += 40;
        });
      }
    }
  };
  std::vector<std::thread> th;
  for (int i = 0; i < std::max(1, nthreads); i++) th.emplace_back(work);
  for (auto& x : th) x.join();
  return 0;
}

// Query stream: terms sampled proportionally to df (query-log-like), distinct
// within a query.  out_terms[q*(max_incl+max_excl) + j]; -1 pads.  nincl/nexcl
// per query are returned in out_nincl/out_nexcl.
int yrwi_synth_queries(const yrwi_synth_cfg* cfg, uint64_t qseed, int32_t nq, int32_t min_incl,
                       int32_t max_incl, int32_t n_excl, int32_t* out_terms, int32_t* out_nincl,
                       int32_t* out_nexcl) {
  Gen g(cfg);
  std::vector<double> cdf((size_t)g.c.n_terms);
  double acc = 0;
  for (int32_t t = 0; t < g.c.n_terms; t++) { acc += (double)g.df[(size_t)t]; cdf[(size_t)t] = acc; }
  int32_t width = max_incl + n_excl;
  for (int32_t q = 0; q < nq; q++) {
    Rng r(hash3(qseed, TAG_Q, (uint64_t)q));
    int32_t ni = min_incl + (int32_t)r.below((uint64_t)(max_incl - min_incl + 1));
    int32_t tot = ni + n_excl;
    std::vector<int32_t> picked;
    int guard = 0;
    while ((int32_t)picked.size() < tot && guard++ < 100000) {
      double x = r.u01() * acc;
      int32_t t = (int32_t)(std::lower_bound(cdf.begin(), cdf.end(), x) - cdf.begin());
      if (t >= g.c.n_terms) t = g.c.n_terms - 1;
      if (std::find(picked.begin(), picked.end(), t) == picked.end()) picked.push_back(t);
    }
    for (int32_t j = 0; j < width; j++) out_terms[(int64_t)q * width + j] = -1;
    for (int32_t j = 0; j < ni; j++) out_terms[(int64_t)q * width + j] = picked[(size_t)j];
    for (int32_t j = 0; j < n_excl; j++) out_terms[(int64_t)q * width + max_incl + j] = picked[(size_t)(ni + j)];
    out_nincl[q] = ni;
    out_nexcl[q] = n_excl;
  }
  return 0;
}

}  // extern "C"
