// yrwi_oracle.cpp -- TEST INFRASTRUCTURE: CPU restatement of YaCy's RWI query
// hot path, used as the parity oracle and as the timed CPU baseline.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
// this library.  The product (yacy_search_server_amd/, libyrwi.so) never does.
//
// Parity pinning: see oracle/README.md.  This file restates, in flat-array
// form, exactly what oracle/java_literal.py restates object-by-object; the
// tests cross-check the two on seeded random cases and on the reference's own
// known-answer tests (SegmentTest, WordReferenceVarsTest, ReferenceContainerTest).
//
// Build: g++ -O2 -std=c++17 -fwrapv -fno-fast-math -ffp-contract=off -shared -fPIC
// (see oracle/Makefile).  Java int/long wrap-around is emulated with explicit
// uint32_t/uint64_t arithmetic, so the file is also UBSan-clean.
//
// Reference citations (paths relative to /root/reference/source/net/yacy):
//   WordReferenceRow.java:49-72 (row), :116-161 (ctor), :241-357 (getters)
//   WordReferenceVars.java:129-158 (from row), :188-209 (clone), :287-294
//     (distance), :301-322 (toRowEntry), :357-361 (virtualAge), :383-455
//     (min/max), :465-499 (join), :534-537 (addPosition)
//   AbstractReference.java:40-60 (distance from positions)
//   ReferenceContainer.java:310-571 (join/exclude algebra)
//   AbstractIndex.java:96-128, TermSearch.java:42-70 (term lookup rules)
//   ReferenceOrder.java:163-216 (normalise, authority), :223-265 (cardinal)
//   WeakPriorityBlockingQueue.java:119-134, :414-425 (bounded top-k order)
//   ByteArray.java:80-84, MicroDate.java:37-55, Base64Order.java:38,533-553,
//   DigestURL.java:352-374, Bitfield.java:88-93, Tokenizer.java:51-56

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

// ---------------------------------------------------------------- Java ints
inline int32_t i32(int64_t x) { return (int32_t)(uint32_t)(uint64_t)x; }
inline int32_t add32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
inline int32_t sub32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
inline int32_t mul32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
inline int32_t shl32(int32_t a, int32_t n) { return (int32_t)((uint32_t)a << (n & 31)); }
inline int32_t div32(int32_t a, int32_t b) {  // Java int division (b != 0)
  if (b == -1) return (int32_t)(0u - (uint32_t)a);
  return a / b;
}
inline int64_t add64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int32_t d2i(double d) {  // Java (int) cast
  if (d != d) return 0;
  if (d >= 2147483647.0) return 2147483647;
  if (d <= -2147483648.0) return (int32_t)0x80000000u;
  return (int32_t)d;
}

// ------------------------------------------------------------- Base64Order
int8_t AHPLA[256];
const char* ALPHA = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
struct AhplaInit {
  AhplaInit() {
    for (int i = 0; i < 256; i++) AHPLA[i] = -1;
    for (int i = 0; i < 64; i++) AHPLA[(uint8_t)ALPHA[i]] = (int8_t)i;
  }
} ahpla_init;

struct Key {  // 72-bit key: hi = bits 71..8, lo = bits 7..0
  uint64_t hi;
  uint32_t lo;
  bool operator<(const Key& o) const { return hi < o.hi || (hi == o.hi && lo < o.lo); }
  bool operator==(const Key& o) const { return hi == o.hi && lo == o.lo; }
};

inline Key key_of(const uint8_t* h) {
  uint64_t hi = 0;
  for (int j = 0; j < 10; j++) hi = (hi << 6) | (uint64_t)AHPLA[h[j]];
  uint32_t c10 = (uint32_t)AHPLA[h[10]], c11 = (uint32_t)AHPLA[h[11]];
  hi = (hi << 4) | (c10 >> 2);
  uint32_t lo = ((c10 & 3u) << 6) | c11;
  return Key{hi, lo};
}

inline bool wellformed(const uint8_t* h) {
  for (int j = 0; j < 12; j++)
    if (AHPLA[h[j]] < 0) return false;
  return true;
}

inline int32_t bytearray_hashcode(const uint8_t* h, int n) {
  int32_t x = 0;
  for (int j = 0; j < n; j++) x = add32(mul32(31, x), (int32_t)h[j]);
  return x;
}

// ---------------------------------------------------------------- MicroDate
const int64_t DAY = 86400000LL;
inline int32_t micro_date_days(int64_t ms) { return (int32_t)((ms / DAY) % 262144LL); }
inline int64_t reverse_micro_date_days(int64_t days, int64_t now_ms) {
  int64_t v = (int64_t)((uint64_t)days * (uint64_t)DAY);
  return std::min(now_ms, v);
}

// ------------------------------------------------------------ row columns
enum {
  OFF_H = 0, OFF_A = 12, OFF_S = 14, OFF_U = 16, OFF_W = 17, OFF_P = 19, OFF_D = 21,
  OFF_L = 22, OFF_X = 24, OFF_Y = 25, OFF_M = 26, OFF_N = 27, OFF_G = 28, OFF_Z = 29,
  OFF_C = 33, OFF_T = 34, OFF_R = 36, OFF_O = 37, OFF_I = 38, OFF_K = 39, ROW = 40
};
inline int u16be(const uint8_t* r, int off) { return ((int)r[off] << 8) | (int)r[off + 1]; }
inline void put16(uint8_t* r, int off, int32_t v) { r[off] = (uint8_t)(v >> 8); r[off + 1] = (uint8_t)v; }

// ---------------------------------------------------------- WordReferenceVars
struct Vars {
  const uint8_t* h;  // url hash (12)
  int urllength, urlcomps, wordsintitle, hitcount, wordsintext, phrasesintext;
  int posintext, posinphrase, posofphrase, llocal, lother;
  int64_t lastModified;
  int32_t virtualAge;
  uint8_t lang[2];
  bool lang_null;
  uint8_t type;
  uint8_t flags[4];
  int32_t distance_field;
  bool has_pos;  // in the row path a Vars holds at most one joined position
  int32_t pos;
  double tf;

  static Vars from_row(const uint8_t* r, int64_t now_ms) {  // Vars(WordReferenceRow) :129-158
    Vars v;
    v.h = r + OFF_H;
    v.urllength = r[OFF_M];
    v.urlcomps = r[OFF_N];
    v.wordsintitle = r[OFF_U];
    v.hitcount = r[OFF_C];
    v.wordsintext = u16be(r, OFF_W);
    v.phrasesintext = u16be(r, OFF_P);
    v.posintext = u16be(r, OFF_T);
    v.posinphrase = r[OFF_R];
    v.posofphrase = r[OFF_O];
    v.llocal = r[OFF_X];
    v.lother = r[OFF_Y];
    v.lastModified = reverse_micro_date_days(u16be(r, OFF_A), now_ms);
    v.virtualAge = u16be(r, OFF_A);
    v.lang[0] = r[OFF_L];
    v.lang[1] = r[OFF_L + 1];
    v.lang_null = (r[OFF_L] == 0 && r[OFF_L + 1] == 0);
    v.type = r[OFF_D];
    std::memcpy(v.flags, r + OFF_Z, 4);
    v.distance_field = r[OFF_I];
    v.has_pos = false;
    v.pos = 0;
    v.tf = (double)v.hitcount / (double)(v.wordsintext + v.wordsintitle + 1);
    return v;
  }

  Vars clone() const {  // 18-arg ctor: distance = 0, virtualAge = -1 (:116, :122)
    Vars c = *this;
    c.distance_field = 0;
    c.virtualAge = -1;
    return c;
  }

  int32_t abstract_distance() const {  // AbstractReference.distance :40-60 (one position)
    if (!has_pos) return 0;
    int32_t d = 0;
    if (posintext > 0) d = std::abs(sub32(posintext, pos));
    return d;  // d == 0 ? 0 : d / 1
  }
  int32_t distance() const {  // :287-294
    int32_t v = abstract_distance();
    return v == 0 ? distance_field : v;
  }
  int32_t virtual_age() {  // :357-361
    if (virtualAge > 0) return virtualAge;
    virtualAge = micro_date_days(lastModified);
    return virtualAge;
  }
  double term_frequency() {  // :374-377
    if (tf == 0.0) tf = (double)hitcount / (double)(wordsintext + wordsintitle + 1);
    return tf;
  }
  void add_position(int32_t p) {  // :534-537 (only ever called once per Vars in the row path)
    if (p > 0) { has_pos = true; pos = p; }
  }

  void min_with(Vars& o) {  // :383-418
    if (hitcount > o.hitcount) hitcount = o.hitcount;
    if (llocal > o.llocal) llocal = o.llocal;
    if (lother > o.lother) lother = o.lother;
    { int32_t v = o.virtual_age(); if (virtual_age() > v) virtualAge = v; }
    if (wordsintext > o.wordsintext) wordsintext = o.wordsintext;
    if (phrasesintext > o.phrasesintext) phrasesintext = o.phrasesintext;
    if (posintext > o.posintext) posintext = o.posintext;
    if (distance() > 0 || o.distance() > 0) {
      int32_t odist = o.distance(), dist = distance();
      if (odist > 0 && odist < dist) { has_pos = true; pos = add32(posintext, odist); }
    }
    if (posinphrase > o.posinphrase) posinphrase = o.posinphrase;
    if (posofphrase > o.posofphrase) posofphrase = o.posofphrase;
    if (lastModified > o.lastModified) lastModified = o.lastModified;
    if (urllength > o.urllength) urllength = o.urllength;
    if (urlcomps > o.urlcomps) urlcomps = o.urlcomps;
    if (wordsintitle > o.wordsintitle) wordsintitle = o.wordsintitle;
    if (tf > o.tf) tf = o.tf;
  }

  void max_with(Vars& o) {  // :420-455
    if (hitcount < o.hitcount) hitcount = o.hitcount;
    if (llocal < o.llocal) llocal = o.llocal;
    if (lother < o.lother) lother = o.lother;
    { int32_t v = o.virtual_age(); if (virtual_age() < v) virtualAge = v; }
    if (wordsintext < o.wordsintext) wordsintext = o.wordsintext;
    if (phrasesintext < o.phrasesintext) phrasesintext = o.phrasesintext;
    if (posintext < o.posintext) posintext = o.posintext;
    if (distance() > 0 || o.distance() > 0) {
      int32_t odist = o.distance(), dist = distance();
      if (odist > 0 && odist > dist) { has_pos = true; pos = add32(posintext, odist); }
    }
    if (posinphrase < o.posinphrase) posinphrase = o.posinphrase;
    if (posofphrase < o.posofphrase) posofphrase = o.posofphrase;
    if (lastModified < o.lastModified) lastModified = o.lastModified;
    if (urllength < o.urllength) urllength = o.urllength;
    if (urlcomps < o.urlcomps) urlcomps = o.urlcomps;
    if (wordsintitle < o.wordsintitle) wordsintitle = o.wordsintitle;
    if (tf < o.tf) tf = o.tf;
  }

  void join(Vars& oe) {  // :465-499
    if (posintext > 0 && oe.posintext > 0) {
      if (posintext > oe.posintext) {
        add_position(posintext);
        posintext = oe.posintext;
      } else {
        add_position(oe.posintext);
      }
    } else if (posintext == 0) {
      posintext = oe.posintext;
    }
    int oe_pop = oe.posofphrase;
    if (posofphrase == oe_pop) {
      posinphrase = std::min(posinphrase, oe.posinphrase);
    } else if (posofphrase > oe_pop) {
      posofphrase = oe_pop;
      posinphrase = oe.posinphrase;
    }
    tf = tf + oe.term_frequency();
    wordsintext = std::max(wordsintext, oe.wordsintext);
    wordsintitle = std::max(wordsintitle, oe.wordsintitle);
    phrasesintext = std::max(phrasesintext, oe.phrasesintext);
    hitcount = std::max(hitcount, oe.hitcount);
  }

  // toRowEntry (:301-322) -> WordReferenceRow ctor (WordReferenceRow.java:116-161)
  bool to_row(uint8_t* out, int64_t now_ms) const {
    if (lang_null) return false;  // ASCII.getBytes(null) -> NullPointerException
    int32_t mddlm = micro_date_days(lastModified);
    int32_t mddct = micro_date_days(now_ms);
    std::memcpy(out + OFF_H, h, 12);
    put16(out, OFF_A, mddlm);
    put16(out, OFF_S, std::max(0, add32(mddlm, mul32(sub32(mddct, mddlm), 2))));
    out[OFF_U] = (uint8_t)wordsintitle;
    put16(out, OFF_W, wordsintext);
    put16(out, OFF_P, phrasesintext);
    out[OFF_D] = type;
    out[OFF_L] = lang[0];
    out[OFF_L + 1] = lang[1];
    out[OFF_X] = (uint8_t)llocal;
    out[OFF_Y] = (uint8_t)lother;
    out[OFF_M] = (uint8_t)urllength;
    out[OFF_N] = (uint8_t)urlcomps;
    out[OFF_G] = 0;
    std::memcpy(out + OFF_Z, flags, 4);
    out[OFF_C] = (uint8_t)hitcount;
    put16(out, OFF_T, posintext);
    out[OFF_R] = (uint8_t)posinphrase;
    out[OFF_O] = (uint8_t)posofphrase;
    out[OFF_I] = (uint8_t)distance();
    out[OFF_K] = 0;
    return true;
  }
};

// -------------------------------------------------------------- containers
struct Container {
  std::vector<uint8_t> rows;  // owned copy (joined results)
  const uint8_t* ext = nullptr;  // or a view of an input list
  int64_t n = 0;
  const uint8_t* row(int64_t i) const { return (ext ? ext : rows.data()) + i * ROW; }
  Key key(int64_t i) const { return key_of(row(i)); }
};

inline int log2j(int32_t x) {  // ReferenceContainer.log2 :391-395
  int l = 0;
  while (x > 0) { x >>= 1; l++; }
  return l;
}

struct Err {
  int code = 0;
  std::string msg;
};

// joinConstructive dispatch :406-416
inline bool dispatch_by_test(int64_t n1, int64_t n2, bool* small_is_i1) {
  int32_t s1 = (int32_t)n1, s2 = (int32_t)n2;
  int32_t high = s1 > s2 ? s1 : s2, low = s1 > s2 ? s2 : s1;
  int32_t steps_enum = mul32(10, sub32(add32(high, low), 1));
  int32_t steps_test = mul32(mul32(12, log2j(high)), low);
  *small_is_i1 = s1 < s2;
  return steps_enum > steps_test;
}

bool join_by_test(const Container& small, const Container& large, int32_t maxd, int64_t now_ms,
                  Container* out, Err* err) {
  out->rows.clear();
  int64_t j = 0;
  for (int64_t i = 0; i < small.n; i++) {
    Key k = small.key(i);
    // binary search in large (RowSet.binarySearch); small is sorted so the
    // search window can start at the previous hit
    int64_t lo = j, hi = large.n;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if (large.key(mid) < k) lo = mid + 1; else hi = mid;
    }
    j = lo;
    if (lo < large.n && large.key(lo) == k) {
      Vars ie2 = Vars::from_row(large.row(lo), now_ms);
      Vars ie1 = Vars::from_row(large.row(lo), now_ms);  // self-join (:440-441)
      ie1.join(ie2);
      if (ie1.distance() <= maxd) {
        size_t o = out->rows.size();
        out->rows.resize(o + ROW);
        if (!ie1.to_row(out->rows.data() + o, now_ms)) {
          err->code = -7; err->msg = "row with empty language cell (reference NPE)";
          return false;
        }
      }
    }
  }
  out->n = (int64_t)(out->rows.size() / ROW);
  out->ext = nullptr;
  return true;
}

bool join_by_enum(const Container& i1, const Container& i2, int32_t maxd, int64_t now_ms,
                  Container* out, Err* err) {
  out->rows.clear();
  int64_t p1 = 0, p2 = 0;
  if (i1.n > 0 && i2.n > 0) {
    while (true) {
      Key k1 = i1.key(p1), k2 = i2.key(p2);
      if (k1 < k2) {
        if (++p1 >= i1.n) break;
      } else if (k2 < k1) {
        if (++p2 >= i2.n) break;
      } else {
        Vars ie1 = Vars::from_row(i1.row(p1), now_ms);
        Vars ie2 = Vars::from_row(i2.row(p2), now_ms);
        ie1.join(ie2);
        if (ie1.distance() <= maxd) {
          size_t o = out->rows.size();
          out->rows.resize(o + ROW);
          if (!ie1.to_row(out->rows.data() + o, now_ms)) {
            err->code = -7; err->msg = "row with empty language cell (reference NPE)";
            return false;
          }
        }
        if (++p1 >= i1.n) break;
        if (++p2 >= i2.n) break;
      }
    }
  }
  out->n = (int64_t)(out->rows.size() / ROW);
  out->ext = nullptr;
  return true;
}

}  // namespace

// ============================================================== C ABI
extern "C" {

typedef struct yo_profile {  // RankingProfile public fields, RankingProfile.java:81-88 order
  int32_t coeff_domlength, coeff_date, coeff_wordsintitle, coeff_wordsintext, coeff_phrasesintext,
      coeff_llocal, coeff_lother, coeff_urllength, coeff_urlcomps, coeff_hitcount,
      coeff_posintext, coeff_posofphrase, coeff_posinphrase, coeff_authority, coeff_worddistance,
      coeff_appurl, coeff_app_dc_title, coeff_app_dc_creator, coeff_app_dc_subject,
      coeff_app_dc_description, coeff_appemph, coeff_catindexof, coeff_cathasimage,
      coeff_cathasaudio, coeff_cathasvideo, coeff_cathasapp, coeff_urlcompintoplist,
      coeff_descrcompintoplist, coeff_prefer, coeff_termfrequency, coeff_language,
      coeff_citation;
} yo_profile;

typedef struct yo_hit {
  uint8_t urlhash[12];
  int32_t tiebreak;  // ByteArray.hashCode(urlhash)
  int64_t score;     // ReferenceOrder.cardinal
} yo_hit;

typedef struct yo_list {
  const uint8_t* term;  // 12-byte term hash
  const uint8_t* rows;  // n sorted 40-byte rows, or NULL if the term is unknown
  int64_t n;
} yo_list;

// Normalisation state after the canonical fold (diagnostics / GPU cross-checks).
typedef struct yo_norm {
  int32_t min_f[13], max_f[13];  // see field order in yo_norm_fields()
  double min_tf, max_tf;
  int32_t max_distance_D;
  int32_t maxdomcount;
  int64_t m;
} yo_norm;

typedef struct yo_trace {
  int32_t nsteps;
  int32_t by_test[3];
  int64_t n1[3], n2[3], nout[3];
} yo_trace;

const char* yo_norm_fields(void) {
  return "hitcount,llocal,lother,virtualAge,wordsintext,phrasesintext,posintext,posinphrase,"
         "posofphrase,urllength,urlcomps,wordsintitle,distance";
}

void yo_profile_default(yo_profile* p) {  // RankingProfile(TEXT) :90-125
  std::memset(p, 0, sizeof(*p));
  p->coeff_appemph = 5; p->coeff_appurl = 12; p->coeff_app_dc_creator = 1;
  p->coeff_app_dc_description = 10; p->coeff_app_dc_subject = 2; p->coeff_app_dc_title = 14;
  p->coeff_authority = 5; p->coeff_date = 9; p->coeff_domlength = 10; p->coeff_hitcount = 1;
  p->coeff_language = 2; p->coeff_llocal = 0; p->coeff_lother = 7; p->coeff_phrasesintext = 0;
  p->coeff_posinphrase = 0; p->coeff_posintext = 4; p->coeff_posofphrase = 0;
  p->coeff_termfrequency = 8; p->coeff_urlcomps = 7; p->coeff_urllength = 6;
  p->coeff_worddistance = 10; p->coeff_wordsintext = 3; p->coeff_wordsintitle = 2;
  p->coeff_urlcompintoplist = 2; p->coeff_descrcompintoplist = 2; p->coeff_prefer = 0;
  p->coeff_citation = 10;
}

// TermSearch + joinExcludeContainers (J1..J7).  Lists may be given in any
// term order; duplicates of a term hash collapse (HandleSet).  Writes the
// joined container (sorted 40-byte rows) to rows_out (capacity `cap` rows).
// Returns 0, or <0 on error (-1 capacity, -2 malformed hash, -7 empty language).
int yo_term_search(const yo_list* incl, int nincl, const yo_list* excl, int nexcl,
                   int32_t max_distance, int64_t now_ms, uint8_t* rows_out, int64_t cap,
                   int64_t* m_out, yo_trace* trace) {
  *m_out = 0;
  if (trace) std::memset(trace, 0, sizeof(*trace));
  // HandleSet semantics: sort by term hash (Base64Order), dedupe.
  auto collect = [](const yo_list* l, int n) {
    std::map<std::pair<uint64_t, uint32_t>, const yo_list*> mp;
    for (int i = 0; i < n; i++) {
      Key k = key_of(l[i].term);
      mp.emplace(std::make_pair(k.hi, k.lo), &l[i]);  // first occurrence kept
    }
    std::vector<const yo_list*> v;
    for (auto& kv : mp) v.push_back(kv.second);
    return v;
  };
  for (int i = 0; i < nincl; i++) if (!wellformed(incl[i].term)) return -2;
  for (int i = 0; i < nexcl; i++) if (!wellformed(excl[i].term)) return -2;
  std::vector<const yo_list*> inc = collect(incl, nincl), exc = collect(excl, nexcl);
  // searchConjunction: any missing/empty term -> empty map (AbstractIndex.java:108-127)
  if (inc.empty()) return 0;
  for (auto* l : inc) if (l->rows == nullptr || l->n == 0) return 0;
  bool use_excl = !exc.empty();
  for (auto* l : exc) if (l->rows == nullptr || l->n == 0) use_excl = false;

  // joinContainers :328-371: TreeMap<(long)(int)(size*1000+count)>; put overwrites.
  std::map<int64_t, const yo_list*> tm;
  for (size_t c = 0; c < inc.size(); c++) {
    int32_t kk = add32(mul32((int32_t)inc[c]->n, 1000), (int32_t)c);
    tm[(int64_t)kk] = inc[c];
  }
  Err err;
  auto it = tm.begin();
  Container acc;
  acc.ext = it->second->rows;
  acc.n = it->second->n;
  ++it;
  int step = 0;
  for (; it != tm.end() && acc.n > 0; ++it) {
    Container nxt;
    nxt.ext = it->second->rows;
    nxt.n = it->second->n;
    bool small_is_i1;
    bool bt = dispatch_by_test(acc.n, nxt.n, &small_is_i1);
    Container res;
    bool ok;
    if (bt) {
      ok = small_is_i1 ? join_by_test(acc, nxt, max_distance, now_ms, &res, &err)
                       : join_by_test(nxt, acc, max_distance, now_ms, &res, &err);
    } else {
      ok = join_by_enum(acc, nxt, max_distance, now_ms, &res, &err);
    }
    if (!ok) return err.code;
    if (trace && step < 3) {
      trace->by_test[step] = bt ? 1 : 0;
      trace->n1[step] = acc.n;
      trace->n2[step] = nxt.n;
      trace->nout[step] = res.n;
      trace->nsteps = step + 1;
    }
    step++;
    acc = std::move(res);
  }
  if (acc.n == 0) return 0;
  // excludeContainers :373-388 -> set difference, order preserving
  std::vector<char> keep((size_t)acc.n, 1);
  if (use_excl) {
    for (auto* l : exc) {
      Container ex;
      ex.ext = l->rows;
      ex.n = l->n;
      int64_t q = 0;
      for (int64_t i = 0; i < acc.n; i++) {
        Key k = acc.key(i);
        while (q < ex.n && ex.key(q) < k) q++;
        if (q < ex.n && ex.key(q) == k) keep[(size_t)i] = 0;
      }
    }
  }
  int64_t m = 0;
  for (int64_t i = 0; i < acc.n; i++) {
    if (!keep[(size_t)i]) continue;
    if (m >= cap) return -1;
    std::memcpy(rows_out + m * ROW, acc.row(i), ROW);
    m++;
  }
  *m_out = m;
  return 0;
}

// normalizeWith (canonical fold) + cardinal for every row of a container.
// scores_out[i] = cardinal(row i).  Returns 0 or <0 (-7 empty language).
int yo_normalize_score(const uint8_t* rows, int64_t m, const yo_profile* prof, const char* lang,
                       int64_t now_ms, int64_t* scores_out, yo_norm* norm_out) {
  if (m <= 0) return 0;
  std::vector<Vars> e((size_t)m);
  for (int64_t i = 0; i < m; i++) {
    e[(size_t)i] = Vars::from_row(rows + i * ROW, now_ms);
    if (e[(size_t)i].lang_null) return -7;
  }
  Vars mn = e[0].clone(), mx = e[0].clone();
  std::unordered_map<uint64_t, int32_t> doms;
  for (int64_t i = 0; i < m; i++) {
    if (i > 0) { mn.min_with(e[(size_t)i]); mx.max_with(e[(size_t)i]); }
    uint64_t hh = 0;
    for (int j = 6; j < 12; j++) hh = (hh << 8) | e[(size_t)i].h[j];
    doms[hh] += 1;
  }
  int32_t maxdom = 0;
  for (auto& kv : doms) maxdom = std::max(maxdom, kv.second);
  const yo_profile& rk = *prof;
  const size_t langlen = std::strlen(lang);
  const double mn_tf = mn.term_frequency(), mx_tf = mx.term_frequency();
  const int32_t mn_va = mn.virtual_age(), mx_va = mx.virtual_age();
  const int32_t mn_d = mn.distance(), mx_d = mx.distance();
  auto inv = [](int32_t t, int32_t lo, int32_t hi, int32_t c) -> int32_t {
    if (hi == lo) return 0;
    return shl32(sub32(256, div32(shl32(sub32(t, lo), 8), sub32(hi, lo))), c);
  };
  auto fwd = [](int32_t t, int32_t lo, int32_t hi, int32_t c) -> int32_t {
    if (hi == lo) return 0;
    return shl32(div32(shl32(sub32(t, lo), 8), sub32(hi, lo)), c);
  };
  auto flag = [](const uint8_t* f, int pos) -> bool { return (f[pos >> 3] & (1 << (pos & 7))) != 0; };
  for (int64_t i = 0; i < m; i++) {
    Vars& t = e[(size_t)i];
    int32_t tfterm = 0;
    if (!(mx_tf == mn_tf))
      tfterm = shl32(d2i(((t.term_frequency() - mn_tf) * 256.0) / (mx_tf - mn_tf)), rk.coeff_termfrequency);
    int dl = (AHPLA[t.h[11]] & 3);
    int32_t dln = dl == 0 ? 4 : dl == 1 ? 10 : dl == 2 ? 14 : 20;  // << (8/20) == << 0
    int32_t r = shl32(sub32(256, dln), rk.coeff_domlength);
    r = add32(r, inv(t.urlcomps, mn.urlcomps, mx.urlcomps, rk.coeff_urlcomps));
    r = add32(r, inv(t.urllength, mn.urllength, mx.urllength, rk.coeff_urllength));
    r = add32(r, inv(t.posintext, mn.posintext, mx.posintext, rk.coeff_posintext));
    r = add32(r, inv(t.posofphrase, mn.posofphrase, mx.posofphrase, rk.coeff_posofphrase));
    r = add32(r, inv(t.posinphrase, mn.posinphrase, mx.posinphrase, rk.coeff_posinphrase));
    r = add32(r, inv(t.distance(), mn_d, mx_d, rk.coeff_worddistance));
    r = add32(r, fwd(t.virtual_age(), mn_va, mx_va, rk.coeff_date));
    r = add32(r, fwd(t.wordsintitle, mn.wordsintitle, mx.wordsintitle, rk.coeff_wordsintitle));
    r = add32(r, fwd(t.wordsintext, mn.wordsintext, mx.wordsintext, rk.coeff_wordsintext));
    r = add32(r, fwd(t.phrasesintext, mn.phrasesintext, mx.phrasesintext, rk.coeff_phrasesintext));
    r = add32(r, fwd(t.llocal, mn.llocal, mx.llocal, rk.coeff_llocal));
    r = add32(r, fwd(t.lother, mn.lother, mx.lother, rk.coeff_lother));
    r = add32(r, fwd(t.hitcount, mn.hitcount, mx.hitcount, rk.coeff_hitcount));
    int64_t R = add64((int64_t)r, (int64_t)tfterm);
    if (rk.coeff_authority > 12) {
      uint64_t hh = 0;
      for (int j = 6; j < 12; j++) hh = (hh << 8) | t.h[j];
      int32_t auth = div32(shl32(doms[hh], 8), add32(1, maxdom));
      R = add64(R, (int64_t)shl32(auth, rk.coeff_authority));
    }
    const int32_t c255 = 255;
    if (flag(t.flags, 28)) R = add64(R, shl32(c255, rk.coeff_appurl));
    if (flag(t.flags, 25)) R = add64(R, shl32(c255, rk.coeff_app_dc_title));
    if (flag(t.flags, 26)) R = add64(R, shl32(c255, rk.coeff_app_dc_creator));
    if (flag(t.flags, 27)) R = add64(R, shl32(c255, rk.coeff_app_dc_subject));
    if (flag(t.flags, 24)) R = add64(R, shl32(c255, rk.coeff_app_dc_description));
    if (flag(t.flags, 29)) R = add64(R, shl32(c255, rk.coeff_appemph));
    if (flag(t.flags, 0)) R = add64(R, shl32(c255, rk.coeff_catindexof));
    if (flag(t.flags, 20)) R = add64(R, shl32(c255, rk.coeff_cathasimage));
    if (flag(t.flags, 21)) R = add64(R, shl32(c255, rk.coeff_cathasaudio));
    if (flag(t.flags, 22)) R = add64(R, shl32(c255, rk.coeff_cathasvideo));
    if (flag(t.flags, 23)) R = add64(R, shl32(c255, rk.coeff_cathasapp));
    if (langlen == 2 && t.lang[0] == (uint8_t)lang[0] && t.lang[1] == (uint8_t)lang[1])
      R = add64(R, shl32(c255, rk.coeff_language));
    scores_out[i] = R;
  }
  if (norm_out) {
    int32_t* a = norm_out->min_f;
    int32_t* b = norm_out->max_f;
    a[0] = mn.hitcount; b[0] = mx.hitcount;
    a[1] = mn.llocal; b[1] = mx.llocal;
    a[2] = mn.lother; b[2] = mx.lother;
    a[3] = mn_va; b[3] = mx_va;
    a[4] = mn.wordsintext; b[4] = mx.wordsintext;
    a[5] = mn.phrasesintext; b[5] = mx.phrasesintext;
    a[6] = mn.posintext; b[6] = mx.posintext;
    a[7] = mn.posinphrase; b[7] = mx.posinphrase;
    a[8] = mn.posofphrase; b[8] = mx.posofphrase;
    a[9] = mn.urllength; b[9] = mx.urllength;
    a[10] = mn.urlcomps; b[10] = mx.urlcomps;
    a[11] = mn.wordsintitle; b[11] = mx.wordsintitle;
    a[12] = mn_d; b[12] = mx_d;
    norm_out->min_tf = mn_tf;
    norm_out->max_tf = mx_tf;
    norm_out->max_distance_D = mx_d;
    norm_out->maxdomcount = maxdom;
    norm_out->m = m;
  }
  return 0;
}

// Bounded top-k in the WeakPriorityBlockingQueue order (score desc, hashCode
// desc); of postings that tie on both, the first in container order wins and
// the later ones are rejected (TreeSet.add returns false).  `maxsize` is the
// queue bound (3000, SearchEvent.java:118); the first k of the queue are output.
int yo_topk(const uint8_t* rows, int64_t m, const int64_t* scores, int32_t maxsize, int32_t k,
            yo_hit* out, int32_t* nout) {
  std::vector<int64_t> idx((size_t)m);
  std::vector<int32_t> hc((size_t)m);
  for (int64_t i = 0; i < m; i++) {
    idx[(size_t)i] = i;
    hc[(size_t)i] = bytearray_hashcode(rows + i * ROW, 12);
  }
  std::sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
    if (scores[a] != scores[b]) return scores[a] > scores[b];
    if (hc[a] != hc[b]) return hc[a] > hc[b];
    return a < b;
  });
  int32_t n = 0;
  int32_t lim = std::min(k, maxsize);
  int64_t prev = -1;
  for (size_t j = 0; j < idx.size() && n < lim; j++) {
    int64_t i = idx[j];
    if (prev >= 0 && scores[prev] == scores[i] && hc[prev] == hc[i]) continue;
    prev = i;
    std::memcpy(out[n].urlhash, rows + i * ROW, 12);
    out[n].tiebreak = hc[(size_t)i];
    out[n].score = scores[i];
    n++;
  }
  *nout = n;
  return 0;
}

// joinConstructive dispatch (:406-416) for arbitrary sizes: 1 = by-test.
int yo_join_dispatch(int64_t n1, int64_t n2, int32_t* small_is_i1) {
  bool s;
  bool bt = dispatch_by_test(n1, n2, &s);
  *small_is_i1 = s ? 1 : 0;
  return bt ? 1 : 0;
}

// joinContainers fold order (:334-366): containers given in term-hash order
// with sizes[i]; writes the fold sequence (indices) to order_out and returns
// its length (TreeMap key collisions drop the earlier container).
int yo_fold_order(const int64_t* sizes, int n, int32_t* order_out) {
  std::map<int64_t, int32_t> tm;
  for (int c = 0; c < n; c++) tm[(int64_t)add32(mul32((int32_t)sizes[c], 1000), (int32_t)c)] = c;
  int k = 0;
  for (auto& kv : tm) order_out[k++] = kv.second;
  return k;
}

// One joinConstructive step (:397-417) with the dispatch given by the caller:
// mode 0 = joinConstructiveByEnumeration(i1, i2) (:448-489), 1 = by test with
// small = i1 / large = i2, 2 = by test with small = i2 / large = i1 (:419-446).
// The sharded protocol (oracle/shard_fold.py) takes the dispatch from the GLOBAL
// container sizes and joins the shard-local rows with it.  Returns 0, -1 when
// `cap` rows are too few, -7 on an empty language cell.
int yo_join_step(const uint8_t* r1, int64_t n1, const uint8_t* r2, int64_t n2, int32_t mode,
                 int32_t max_distance, int64_t now_ms, uint8_t* rows_out, int64_t cap, int64_t* m_out) {
  *m_out = 0;
  Container a, b, res;
  a.ext = r1;
  a.n = n1;
  b.ext = r2;
  b.n = n2;
  Err err;
  bool ok = true;
  if (n1 > 0 && n2 > 0) {
    if (mode == 1) ok = join_by_test(a, b, max_distance, now_ms, &res, &err);
    else if (mode == 2) ok = join_by_test(b, a, max_distance, now_ms, &res, &err);
    else ok = join_by_enum(a, b, max_distance, now_ms, &res, &err);
  }
  if (!ok) return err.code;
  if (res.n > cap) return -1;
  if (res.n > 0) std::memcpy(rows_out, res.rows.data(), (size_t)res.n * ROW);
  *m_out = res.n;
  return 0;
}

// Full canonical query: term search -> normalise -> cardinal -> top-k.
int yo_search(const yo_list* incl, int nincl, const yo_list* excl, int nexcl, int32_t max_distance,
              const yo_profile* prof, const char* lang, int64_t now_ms, int32_t k, yo_hit* out,
              int32_t* nout, yo_norm* norm_out, yo_trace* trace) {
  *nout = 0;
  int64_t cap = 0;
  for (int i = 0; i < nincl; i++) cap = std::max(cap, incl[i].n);
  std::vector<uint8_t> rows((size_t)std::max<int64_t>(cap, 1) * ROW);
  int64_t m = 0;
  int rc = yo_term_search(incl, nincl, excl, nexcl, max_distance, now_ms, rows.data(), cap, &m, trace);
  if (rc != 0) return rc;
  if (norm_out) std::memset(norm_out, 0, sizeof(*norm_out));
  if (m == 0) return 0;
  std::vector<int64_t> sc((size_t)m);
  rc = yo_normalize_score(rows.data(), m, prof, lang, now_ms, sc.data(), norm_out);
  if (rc != 0) return rc;
  return yo_topk(rows.data(), m, sc.data(), 3000, k, out, nout);
}

}  // extern "C"
