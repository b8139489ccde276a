// yrwi_internal.h -- structures shared by the host runtime (yrwi_host.cpp) and
// the gfx950 kernels (yrwi_kernels.hip).  Plain PODs only.
#pragma once

#include <stdint.h>

#include "../../include/yrwi.h"

namespace yrwi {

// ---------------------------------------------------------------- geometry
#ifndef YRWI_JOIN_TILE
#define YRWI_JOIN_TILE 4096
#endif
constexpr int JOIN_TILE = YRWI_JOIN_TILE;  // merge-path items per join workgroup
constexpr int JOIN_THREADS = 256;
constexpr int JOIN_IPT = JOIN_TILE / JOIN_THREADS;
constexpr int JOIN_MAXM = JOIN_TILE / 2 + 1;  // matches per merge tile <= min(#A, #B + 1)

constexpr int CHUNK = 2048;          // container elements per rank/score workgroup
constexpr int CHUNK_THREADS = 256;
constexpr int CHUNK_IPT = CHUNK / CHUNK_THREADS;
constexpr int SEGC = 32;             // fold segments kept per chunk summary
constexpr int SSEG = 128;            // fold segments kept per shard summary
constexpr int NF = 11;               // min/max int fields (virtualAge handled apart)

constexpr int64_t DAY_MS = 86400000LL;

// 72-bit url-hash key (Base64Order.enhancedCoder order == unsigned integer order):
// hi = key >> 8 (chars 0..9 and the top 4 bits of char 10), lo = key & 0xFF.

// A sorted posting list / container on the device (SoA keys + AoS rows).
// uid: the url id of each posting -- its url hash's rank in the context's url
// dictionary (yrwi_dict.hip), so uid order == url-hash order and the joins
// compare and stream 4-byte ids instead of 9-byte keys.  khi/klo (the 72-bit
// key) are kept on index lists only (validation, dictionary build, loader).
struct DList {
  const uint64_t* khi;
  const uint8_t* klo;
  const uint8_t* rows;  // 40-byte WordReferenceRow (index lists; joined containers have none)
  int64_t n;
  const uint32_t* uid;
  const uint64_t* feat;  // FEAT_WORDS words per posting: the ranking record (FeatRec below)
  // line heads of an index list (yrwi_dict.hip, k_heads), nullptr for joined
  // containers: head[g] = uid[32 g] (the first id of every 128-B line of uid),
  // then, at head + head1_cap(n), head[32 g] again every 32nd: uid[1024 g]
  const uint32_t* head;
  // deferred container of a multi-term fold (not its last step): no records, the
  // rows of the fold's lists 0..tw-1 it joins, tw per row (tup[row * tw + list])
  const int32_t* tup;
  int32_t tw;
  // url-id bitmap of a large index list (nullptr: none), 16-B units of
  // BM_UNIT_IDS = 96 ids: 96 bits and the list position of the unit's first id
  // (yrwi_bitmap.h): membership and position of an id in one 16-B load.
  // k_probe looks the smaller side's ids up in it instead of searching the list.
  const uint64_t* bm;
  // words 0-1 of every posting's record (2 per posting; bitmap lists only, else
  // nullptr): the J5 fields k_compact gathers from an enumeration's joined side,
  // 8 postings per 128-B line instead of 4
  const uint64_t* j5;
};
// the two head levels of a list of n postings (each level padded to 32 entries)
__host__ __device__ constexpr int64_t head1_n(int64_t n) { return (n + 31) >> 5; }
__host__ __device__ constexpr int64_t head1_cap(int64_t n) { return (head1_n(n) + 31) & ~(int64_t)31; }
__host__ __device__ constexpr int64_t head2_n(int64_t n) { return (n + 1023) >> 10; }
__host__ __device__ constexpr int64_t heads_cap(int64_t n) { return head1_cap(n) + ((head2_n(n) + 31) & ~(int64_t)31); }

// The ranking record of a posting, 32 bytes (4 little-endian words), built from
// its WordReferenceRow (WordReferenceRow.java:49-72) by k_features and carried
// through every join: the joins gather 32 B of the accumulated side and 16 B of
// the joined side instead of 40-byte rows, and the ranking kernels stream it.
//   w0 = t | w << 16 | p << 32 | u << 48 | c << 56   posintext, wordsintext, phrasesintext, wordsintitle, hitcount
//   w1 = r | o << 8 | i << 16 | x << 24 | y << 32 | m << 40 | n << 48 | d << 56
//        posinphrase, posofphrase, worddistance, llocal, lother, urllength, urlcomps, doctype
//   w2 = a | l << 16 | z << 32          lastModified days, language (byte 22 low), flags (byte 29 low)
//   w3 = h | dl << 32 | host << 34      ByteArray.hashCode(urlhash), domLengthEstimation key (ahpla[urlhash[11]] & 3),
//                                       the url's dense host id in the context (ensure_host_ids; 0 until built)
// The J5 inputs of the joined side (t w p u c r o) are words 0 and 1.
constexpr int FEAT_WORDS = 4;
constexpr int FEAT_BYTES = 8 * FEAT_WORDS;

// Feature rule of a join step (ReferenceContainer.joinConstructive :406-416).
enum JoinMode : int32_t {
  JM_ENUM = 0,        // joinConstructiveByEnumeration: join(Vars(A), B)
  JM_TEST_LARGE_B = 1,// joinConstructiveByTest, small = A (acc), large = B: self-join of B
  JM_TEST_LARGE_A = 2,// joinConstructiveByTest, small = B, large = A: self-join of A
  JM_MARK = 3         // excludeDestructive: mark A rows present in B
};

// Intersection algorithm of a job (independent of the reference's feature rule):
// merge-path tiles for comparable sizes, per-element probing of the large list
// for skewed ones (the galloping bound of BASELINE.md §4).
// JA_BMAND: a counted-only join of two lists that both have url-id bitmaps:
// popcount(bits A & bits B) over ranges of bitmap units (tiles of BMAND_WORDS
// 16-B units), in place of probing one list's ids into the other (k_probe)
// (An AND-of-bitmaps enumeration of two dense lists' matches, JA_BMENUM, was
// built and measured in round 5 -- C2 k_probe 116 -> 164 us, k_compact 228 -> 276:
// its tiles' long match runs left few compaction workgroups -- and removed in
// round 6)
enum JoinAlgo : int32_t { JA_MERGE = 0, JA_PROBE = 1, JA_BMAND = 2 };
constexpr int BMAND_WORDS = 4096;  // 16-B bitmap units per JA_BMAND tile
// url-id bitmap units (DList::bm, yrwi_bitmap.h): 96 ids per 16 B
constexpr int64_t BM_UNIT_IDS = 96;
inline int64_t bm_units(int64_t nurls) { return (nurls + BM_UNIT_IDS - 1) / BM_UNIT_IDS; }
constexpr int PROBE_TILE = 256;  // small-list elements per probe workgroup
#ifndef YRWI_BM_TILE
#define YRWI_BM_TILE 1024
#endif
constexpr int BM_TILE = YRWI_BM_TILE;  // small-list elements per bitmap-probe workgroup (4 per thread; 512: C2 probe 111 -> 150 us)
constexpr int KPT_LARGE = 8;           // ids per thread of a bitmap probe whose small side is long
constexpr int64_t BM_LARGE_MIN = 1 << 18;  // small-side ids from which a bitmap job takes KPT_LARGE

// The lists of a multi-term fold and the join mode of each step, for the last
// step's k_compact: it folds the deferred rows' records (J5/J6 step by step,
// exactly as materialising every step would) before joining the last list.
struct FoldSrc {
  const uint64_t* feat[YRWI_MAX_TERMS];  // ranking records of the fold's lists, in fold order
  const uint64_t* j5[YRWI_MAX_TERMS];    // their DList::j5 (nullptr: none)
  int32_t mode[YRWI_MAX_TERMS];          // JoinMode of step s (lists 0..s with list s+1)
};

// Chained fold (a query of t >= 2 include lists with more lists after its first
// join step: more includes and / or exclusions; no maxDistance filter).  The
// first step (lists 0 and 1) joins as usual; k_chain then tests each of its
// matched pairs against the fold's later include lists and the exclusion lists
// (url-id bitmap: one 16-B word; otherwise the list's ids or line heads around the
// tile's range), keeps only the survivors -- the rows the whole fold and
// exclusion keep, which do not depend on the fold order -- with their rows in the
// later include lists, and k_compact folds their records over all t lists (J5/J6
// step by step, each step's dispatch from the intersection sizes k_chain counts).
// No intermediate container is written.  ReferenceContainer.java:328-388.
constexpr int CHAIN_MAXL = 6;  // lists tested per pair (the url selection, later includes, then exclusions)
constexpr int CHAIN_MAXI = 2;  // later include lists (t <= 4)
constexpr int CHAIN_LVL = 5;   // per-tile counts: matches, after include tests 1, 2, 3, after exclusion
constexpr int CHAIN_GMAX = 32; // tiles of one job per k_chain workgroup (a chain group: int2 {first tile, tiles})
struct ChainList {
  const uint32_t* uid;
  const uint32_t* head;  // line heads (DList::head) or nullptr
  const uint64_t* bm;    // url-id bitmap (DList::bm) or nullptr
  int64_t n;
};
struct ChainQ {
  // include tests first -- the query's url selection (if any: uid = its url ids, no
  // heads, no bitmap), then includes 2..t-1 of the fold (in fold order) -- then
  // the exclusion lists
  ChainList l[CHAIN_MAXL];
  int32_t ninc, nl;          // include tests; all lists
  int32_t pos0, npos;        // the include tests whose row is kept: [pos0, pos0 + npos) (lists 2..t-1)
  int32_t* tup[CHAIN_MAXI];  // each survivor's row in include list 2 + i (slot-indexed like the pairs)
  int64_t* level;            // the job's CHAIN_LVL counts (written by k_scan_tiles; pinned host memory)
  int32_t pre;               // leading include tests done by the first step's probe (JoinQ::chain_bm): 0 or 1
  int32_t perm;              // count-first fold: 1: pairs (row in list 2, row in list 0), tup[0] list 1, tup[1] list 3;
                             // 2 (from list 3): pairs (row in list 3, row in list 0), tup[0] list 1, tup[1] list 2
};

struct ChunkSum;
struct JoinQ {
  DList A, B;
  int64_t tile_base;   // first global tile of this job
  int64_t ntiles;
  int32_t mode;
  int32_t maxd;
  int32_t algo;        // JoinAlgo
  int32_t small_is_A;  // JA_PROBE: which side is probed into the other
  int32_t ptile;       // JA_PROBE: small-list elements per tile (PROBE_TILE, BM_TILE with a bitmap)
  int32_t chained;     // a chained fold's first step (set before layout; JoinQ::chain points at its ChainQ)
  uint8_t* removed;    // JM_MARK target (indexed like A)
  uint32_t* out_uid;   // compacted output container (capacity min(nA, nB))
  uint64_t* out_feat;  // its ranking records (FEAT_WORDS per row)
  int64_t now_ms;
  int64_t* m_out;      // number of output rows (written by the scan kernel)
  // deferred output (out_tw > 0: a step before the fold's last): out_tw source rows
  // per joined row instead of a record; fold: the lists / modes when A is deferred
  int32_t* out_tup;
  int32_t out_tw;
  const FoldSrc* fold;
  // matched pairs of the job: [pair_base, pair_base + cap) of the step's pair
  // arrays; every tile writes its run at tile_src[tile] (merge tiles: the prefix
  // of their bounds min(na, nb + 1); probe tiles: ptile per tile)
  int64_t pair_base;
  const ChainQ* chain;  // chained fold (k_chain, k_compact<true>) or nullptr
  // ChainQ::pre = 1: the first later include list's url-id bitmap, tested by the
  // bitmap probe on its hits before they are written (its rows into chain_tup0,
  // the tile's first two level counts into tile_lvl); chain_fill: level counts
  // 2 and 3 that repeat count 1 (no second later include)
  const uint64_t* chain_bm;
  int32_t* chain_tup0;
  int32_t chain_fill;
  int32_t count_only;  // count the matches (tile_cnt, m_out) and write nothing: a count-first fold's list 0 x 1
  int64_t bm_words;    // JA_BMAND: 16-B bitmap units of the url-id space (bm_units)
  const uint64_t* bm3; // JA_BMAND: a third list's bitmap in the AND (count-first from list 3), or nullptr
  // the query's last step, when the rank phase can take its normalisation pieces
  // from the compaction (no exclusion marks, no authority counts): one ChunkSum per
  // tile of the job (index tile - tile_base), written by k_compact_sum
  ChunkSum* psum;
  int32_t want_sum;    // host: psum wanted (run_join_jobs allocates it)
  int32_t pad_sum;
};

// One merge-path tile of a JA_MERGE job (written by k_partition): the tile's A
// range [a0, a0+na) and B range [b0, b0+nb) plus one lookahead B key (nbl = nb+1
// unless B is exhausted), with direct key pointers so k_join needs no job lookup.
struct TileDesc {
  const uint32_t* a;  // url ids of A and B
  const uint32_t* b;
  int64_t a0, b0;
  int32_t na, nb, nbl, job;
  int32_t maxd, pad;
};
constexpr int TILEDESC_DWORDS = (int)(sizeof(TileDesc) / 4);

// One tile of a JA_PROBE job (written by k_probe_part): the large-list range
// [lo, hi) that holds every key of the tile's PROBE_TILE small-list keys.
struct ProbeDesc {
  int64_t lo, hi;
  int32_t job, pad;
};

// A bitmap-probe tile as k_probe's short path reads it (64 B: one scalar load;
// written by k_probe_part in tile order, copied into the band order by
// k_order_scatter): the smaller list's ids, the larger list's url-id bitmap, the
// tile's first small index and pair slot, its tile index.  BMF_SIMPLE: no
// exclusion mark, distance filter or chain test -- nothing of the job is read.
constexpr int32_t BMF_SIMPLE = 1, BMF_SMALL_A = 2;
struct BmFast {
  const uint32_t* sm_uid;
  const uint64_t* lg_bm;
  int64_t sm_n, s0, src;
  int64_t t;       // the tile (index among the step's probe tiles)
  int32_t flags;   // BMF_*
  int32_t pad[3];
};
static_assert(sizeof(BmFast) == 64, "one 64-B scalar load");

// Per-chunk normalisation summary (ReferenceOrder.NormalizeWorker :163-210,
// restated as an order-preserving reduction).
struct ChunkSum {
  int32_t nvalid;
  int32_t first;        // container index of the first valid element, -1 if none
  int32_t end;          // container index past the summary's last element
  int32_t p_first, od_first, a_first;
  int32_t pmax;         // max posintext over valid elements
  int32_t M_rest, L_rest;  // max / last positive stored distance over the rest
  int32_t mn[NF], mx[NF];  // over all valid elements
  int32_t va_mn_rest, va_mx_rest;  // raw lastModified days over the rest
  int32_t nseg, overflow;
  double tf_mn, tf_mx;
  uint32_t seg[SEGC];   // (P << 16) | (M << 8) | L, in order, P strictly increasing
};

struct ShardSum {
  int32_t nvalid;
  int32_t has_first;
  int32_t p_first, od_first, a_first;
  int32_t mn[NF], mx[NF];
  int32_t va_mn_rest, va_mx_rest;
  int32_t nseg, overflow;
  double tf_mn, tf_mx;
  int32_t maxdom;       // max host count (authority), -1 if not computed
  int32_t pad;
  uint32_t seg[SSEG];
};

struct NormState {
  int32_t mn[NF], mx[NF];
  int32_t va_mn, va_mx;
  int32_t D;            // max.distance() after the fold; min.distance() == 0
  int32_t maxdom;
  int64_t nvalid;
  double tf_mn, tf_mx;
  // fl(1 / divisor) of cardinal's normalisations (0 where max == min): fields
  // [0, NF), then date (va), then worddistance (D) -- see qdiv in yrwi_kernels.hip
  double rcp[NF + 2];
};

// Field indices inside mn/mx.
enum : int {
  F_HITCOUNT = 0, F_LLOCAL, F_LOTHER, F_WORDSINTEXT, F_PHRASESINTEXT, F_POSINTEXT,
  F_POSINPHRASE, F_POSOFPHRASE, F_URLLENGTH, F_URLCOMPS, F_WORDSINTITLE
};

// Device copy of a query's yrwi_filter (SearchEvent.addRWIs constraints).
struct FilterQ {
  uint8_t constraint[4];
  int32_t has_constraint, all_of;
  int32_t contentdom, strict;
  uint8_t lang[8];
  int32_t lang_len;          // 0: any language
  int32_t has_site, has_alt;
  uint64_t site, altsite;    // 36-bit host keys (alphabet index per char of url-hash chars 6..11)
  const uint64_t* siteex;    // sorted host keys
  int64_t nsiteex;
  const uint64_t* url_hi;    // sorted url keys of the doublecheck set
  const uint8_t* url_lo;
  int64_t nurl;
  int32_t* flagcount;        // 32 device counters or nullptr
};

struct RankQ {
  const uint64_t* feat;    // container ranking records (sorted by url hash), FEAT_WORDS per element
  const uint32_t* uid;     // container url ids (keys from the url dictionary dkhi/dklo) ...
  const uint64_t* ekhi;    // ... or, without url ids, the elements' own keys
  const uint8_t* eklo;
  const uint64_t* dkhi;    // url dictionary: key of every url id
  const uint8_t* dklo;
  const uint8_t* removed;  // exclusion marks or nullptr
  int64_t n;
  int64_t chunk_base;
  int64_t nchunks;
  yrwi_profile prof;
  uint8_t lang[2];
  int32_t lang_ok;         // target language has exactly 2 chars
  int64_t now_ms;
  int32_t k;
  int32_t want_authority;  // coeff_authority > 12
  uint64_t* hkeys;         // authority host table (open addressing), nullptr if unused
  uint32_t* hcnt;
  uint64_t hmask;
  uint32_t idx_tag;        // shard << 28, OR-ed into candidate indices
  int32_t kout;            // results wanted (k is the stack bound: 3000 with doubledom)
  const FilterQ* filt;     // addRWIs constraints or nullptr
  int32_t doubledom;       // results in pullOneRWI(skipDoubleDom) order
  int32_t host_rec;        // the records carry their url's dense host id (w3 >> 34): the host tables key on it
  int32_t hp_nb;           // authority by partition (ecnt): the query's host buckets
  int32_t* ecnt;           // ... and every element's host count (nullptr: the host tables serve)
  int64_t hp_hoff;         // ... its first histogram entry (bucket-major: hp_hoff + bucket * nchunks + chunk)
  int32_t* hp_hist;        // ... the histogram (k_reduce counts every chunk's buckets into it)
  // normalisation pieces written by the compaction (JoinQ::psum), in container
  // order, or nullptr: k_reduce skips the query; k_piece_merge merges them 64 at a
  // time into groups, which k_shard_fin folds instead of chunk summaries
  const ChunkSum* pieces;
  int64_t npieces;
  ChunkSum* groups;
  int64_t ngroups;
};

struct Cand {  // top-k candidate: sort descending on (k1, k2)
  uint64_t k1;  // score ^ 2^63
  uint64_t k2;  // ((hashCode ^ 2^31) << 32) | ~index
};

// host-count exchange between url-hash shards (authority, ReferenceOrder.java:176-216)
struct HostMsg {
  uint64_t key;  // host hash (url-hash chars 6..11, 36 bits) + 1
  uint32_t q;    // query index in the batch
  uint32_t cnt;  // count of that host in the sender's part of the joined container
};

// ---------------------------------------------------------------- launchers
// host -> device copies of up to COPY_IN_MAX staged ranges in one launch: src =
// device address of pinned host memory, dst = device memory (yrwi_host.h upload)
constexpr int COPY_IN_MAX = 8;
struct CopyIn {
  const uint8_t* src[COPY_IN_MAX];
  uint8_t* dst[COPY_IN_MAX];
  uint64_t bytes[COPY_IN_MAX];
  int32_t n;
};
int launch_copy_in(const CopyIn& c, void* stream);
// device -> pinned host readback (dst: device address of pinned host memory): n
// elements of `elem` bytes, the source's `stride` bytes apart (4-B words when aligned)
int launch_gather_out(uint8_t* dst, const uint8_t* src, int64_t n, int32_t elem, int64_t stride, void* stream);
// host_key (nullptr: the tables hold host hashes): the tables hold dense host ids + 1, host_key[id] = host hash
int launch_host_count(const uint64_t* hkeys, int64_t nslots, int world, uint32_t* owner_cnt, void* stream,
                      const uint64_t* host_key = nullptr);
int launch_host_pack(const uint64_t* hkeys, const uint32_t* hcnt, const int64_t* slot_base, int nq, int64_t nslots,
                     int world, uint32_t* cursor, HostMsg* send, uint64_t* send_slot, void* stream,
                     const uint64_t* host_key = nullptr);
int launch_host_owner(const HostMsg* recv, int64_t nrecv, uint64_t* okeys, uint32_t* ocnt, uint64_t omask,
                      int32_t* gmax, uint32_t* reply, void* stream);
int launch_host_apply(const uint32_t* back, const uint64_t* send_slot, int64_t n, uint32_t* hcnt_all,
                      ShardSum* ss, const int32_t* gmax, int nq, void* stream);
// (defined in yrwi_kernels.hip; all asynchronous on `stream`)
int launch_validate_rows(const uint8_t* rows, int64_t n, uint64_t* khi, uint8_t* klo, int32_t* err,
                         void* stream);
// ranking records (FeatRec) of n rows
int launch_features(const uint8_t* rows, int64_t n, uint64_t* feat, void* stream);
// joined container -> 40-byte rows as toRowEntry writes them (WordReferenceVars.java:301-327):
// key of url id uid[i] from the dictionary, the record's columns, freshUntil from "now"
int launch_feat_rows(const uint64_t* feat, const uint32_t* uid, const uint64_t* dkhi, const uint8_t* dklo, int64_t n,
                     int64_t now_ms, uint8_t* rows, void* stream);
// Band-major schedules of a join step (k_order_hist and k_order_scatter in
// yrwi_kernels.hip).  Compaction: the url id each tile starts at (key, one per
// tile), band = key >> shift, the tiles in that order (perm: tile, job).
// Probe: 16 url-id bands per probe tile (pkey = first id >> pshift), the probe
// tiles in that order (pperm; tile index relative to the first probe tile).  key / pkey == nullptr: job order.  tile_job (any
// order) spares k_compact a search of the job table per tile.
struct BandOrder {
  int32_t* tile_job = nullptr;  // job of every tile (k_partition / k_probe_part; k_compact reads it)
  uint32_t* key = nullptr;
  int2* perm = nullptr;
  uint32_t* pkey = nullptr;
  int2* pperm = nullptr;
  int32_t* hist = nullptr;      // bucket counts of both sorts' workgroups (scratch, ORDER_HIST_SLICES x 4096)
  int32_t shift = 0, pshift = 0;
};
constexpr int ORDER_SLICE_MIN = 2048;  // tiles per counting-sort workgroup (at most 64 per order)
constexpr int ORDER_HIST_SLICES = 128;
struct OrderProb {
  const uint32_t* key;
  int64_t n, slice;
  int32_t shift, nslices;
  const int32_t* tile_job;
  int2* perm;
  int32_t* hist;
  const BmFast* pay;  // rows copied into the order beside perm (nullptr: none)
  BmFast* pay_out;
};
struct OrderArgs {
  OrderProb p[2];
};

// jobs [0, nmerge) are JA_MERGE with tiles [0, merge_tiles); the rest are JA_PROBE
// chain: the step has chained jobs (JoinQ::chain): k_chain and k_scan_tiles run
// (d_tile_lvl: CHAIN_LVL counts per tile), k_compact does not -- the caller
// launches it with launch_compact once the fold's dispatch modes are known
int launch_join_step(const JoinQ* d_jobs, const int64_t* d_tile_base, int32_t njobs, int32_t nmerge,
                     int64_t merge_tiles, int64_t total_tiles, TileDesc* d_desc, ProbeDesc* d_pdesc,
                     uint2* d_pairs, uint32_t* d_pair_uid, int64_t* d_tile_src,
                     int32_t* d_tile_cnt, int64_t* d_tile_off, bool mark, bool long_tiles, const BandOrder& bo,
                     void* stream,
                     void* ev_begin,
                     void* ev_mid, void* ev_end, void* ev_compact0 = nullptr, void* ev_compact1 = nullptr,
                     bool chain = false, int32_t* d_tile_lvl = nullptr, ProbeDesc* d_crange = nullptr,
                     const int2* d_cgrp = nullptr, int64_t ngroups = 0, BmFast* d_fast = nullptr,
                     BmFast* d_fast_perm = nullptr, int sum = 0);
// sum: jobs of the step with normalisation pieces (JoinQ::psum), compacted by
// k_compact_sum (one wave per tile): 0 none, 1 every job, 2 some (k_compact the rest)
int launch_compact(const JoinQ* d_jobs, const int64_t* d_tile_base, int32_t njobs, int64_t total_tiles,
                   const uint2* d_pairs, const uint32_t* d_pair_uid, const int64_t* d_tile_src,
                   const int32_t* d_tile_cnt, const int64_t* d_tile_off, const BandOrder& bo, bool chain, void* stream,
                   int sum = 0);
int launch_rank(const RankQ* d_q, const int64_t* d_chunk_base, int32_t nq, int64_t total_chunks,
                ChunkSum* d_chunks, ShardSum* d_shard, NormState* d_norm, int32_t world, void* stream);
// hp_any: some query of the launch counts host buckets (RankQ::ecnt): k_reduce
// then takes HPART_MAXS ints of dynamic LDS for them (the others launch without)
// reduce: some query of the launch has no normalisation pieces (RankQ::pieces) --
// without one k_reduce is not launched
// group_q / ngroups: (query, group) of every group of merged pieces (k_piece_merge)
int launch_reduce(const RankQ* d_q, const int64_t* d_chunk_base, const int32_t* d_chunk_q, int32_t nq,
                  int64_t total_chunks,
                  ChunkSum* d_chunks, ShardSum* d_shard, void* stream, void* ev_mid = nullptr, bool hp_any = false,
                  bool reduce = true, const int2* d_group_q = nullptr, int64_t ngroups = 0);
// authority host counts by partition (RankQ::ecnt): histogram per (query bucket, chunk) -> scan ->
// scatter (host id, element) -> per-bucket LDS counts, every element's count, maxdomcount
int launch_host_part(const RankQ* d_q, const int32_t* d_chunk_q, int64_t total_chunks, int32_t* d_hist,
                     int32_t* d_hoffs, int64_t nhist, void* d_tmp, size_t tmp_bytes, uint2* d_part, const int2* d_bq,
                     int32_t nbuckets, ShardSum* d_shard, void* stream);
size_t host_part_tmp_bytes(int64_t nhist);  // scan scratch for nhist + 1 histogram entries
constexpr int HPART_MAXS = 1024, HPART_TARGET = 512;  // buckets per query at most; elements per bucket aimed at
int launch_combine(const RankQ* d_q, int32_t nq, const ShardSum* d_shards, int32_t world,
                   NormState* d_norm, void* stream);
// chunks in d_order ((chunk, query) int pairs); d_tq: per-query score threshold (zeroed), see PruneP in yrwi_kernels.hip
int launch_score(const RankQ* d_q, const int32_t* d_chunk_q, const int32_t* d_order, int32_t nq, int64_t total_chunks,
                 int64_t seed_chunks, const NormState* d_norm, Cand* d_cand, int32_t* d_cand_cnt, int32_t kc,
                 int32_t* d_redo, int32_t* d_nredo, unsigned long long* d_tq, void* d_qtab, void* stream,
                 void* ev_mid = nullptr);
size_t score_qtab_bytes();  // per query: d_qtab of launch_score (its pruning parameters and term tables)
// candidates one k_topq group may hold (lists per group = min(64, capacity / list stride))
int topq_capacity(int32_t keff);
// top-k of candidate-list groups: group g = lists [gbase[g], gbase[g]+gn[g]) of d_in (stride
// in_stride, counts d_in_cnt), k = gk[g]; output list g at d_out + g*keff, count d_out_cnt[g]
int launch_topq(const int64_t* d_gbase, const int32_t* d_gn, const int32_t* d_gk, int64_t ngroups, const Cand* d_in,
                const int32_t* d_in_cnt, int32_t in_stride, int32_t keff, Cand* d_out, int32_t* d_out_cnt, void* stream);
// mode 0: first kout hits of the non-doubledom queries; 1: every query's stack
// (k hits); 2: only the doubledom queries' stacks
int launch_emit(const RankQ* d_q, int32_t nq, const Cand* const* d_final, const int32_t* const* d_final_cnt,
                int32_t kmax, yrwi_hit* d_hits, int32_t* d_nout, int mode, void* stream);
// out[i] = sum or max over r of all[r * n + i] (loopback allreduce)
int launch_reduce_i32(const int32_t* all, int world, int64_t n, int32_t* out, int max_op, void* stream);
// results from stacks (stride kint): pullOneRWI(skipDoubleDom) order for doubledom
// queries, the first kout entries for the others (only_dd: doubledom queries only)
int launch_pull(const RankQ* d_q, int32_t nq, const yrwi_hit* d_stack, const int32_t* d_scnt, int32_t kint,
                int only_dd, int32_t kmax, yrwi_hit* d_hits, int32_t* d_nout, void* stream);
// merge of gathered shard stacks allh[world][nq][kint] into stack[nq][kint] (TreeSet in shard order)
int launch_gmerge(const RankQ* d_q, const yrwi_hit* d_allh, const int32_t* d_alln, int world, int32_t nq, int32_t kint,
                  uint32_t* d_slot, uint8_t* d_dup, yrwi_hit* d_stack, int32_t* d_scnt, void* stream);
// cardinal(URIMetadataNode) of n node records
int launch_score_nodes(const yrwi_node* d_nodes, int64_t n, const yrwi_profile* d_prof, const char* lang8,
                       int32_t maxdomcount, int64_t* d_scores, void* stream);
int launch_score_all(const RankQ* d_q, const int32_t* d_chunk_q, int32_t nq, int64_t total_chunks,
                     const NormState* d_norm, int64_t* d_scores, void* stream);

// ------------------------------------------------ search events
// A SearchEvent that receives containers one after another (the local RWI
// process and every remote peer, SearchEvent.addRWIs :673-836 from
// RWIProcess.run and Protocol.remoteSearchProcess :802): normalisation state,
// host counts, the doublecheck url set, the flag counts and the rwiStack persist
// across arrivals in device memory.
constexpr int EV_THREADS = 256;
constexpr int EV_CH = 1024;    // arrival rows per chunk (4 per thread)
constexpr int EV_SUBS = 512;   // url-set sub-tables (9 key bits select one, see uset_slot)

struct EvState {
  int32_t started;             // ReferenceOrder.min/max exist
  int32_t P, A, hasA;          // max-distance fold
  int32_t mn[NF], mx[NF];
  int32_t va_mn, va_mx;
  int32_t maxdom;              // ReferenceOrder.maxdomcount
  int32_t nstack, cur;         // stack entries, current stack half
  int32_t epoch;               // non-empty arrivals applied
  int32_t err;                 // YRWI_E_* once a table overflowed (event unusable)
  int32_t pad;
  int32_t flagcount[32];       // SearchEvent.flagcount
  int64_t nin, nadmit_local, nadmit_remote, nremote;
  double tf_mn, tf_mx;
};

struct EvDev {
  RankQ q;          // prof, lang, now_ms, want_authority, host table (hkeys/hcnt/hmask), k = stack bound
  FilterQ f;        // addRWIs constraints (doublecheck seeds live in the url set)
  int32_t has_filter, ulog;
  EvState* st;
  uint64_t* ukey;   // url set: EV_SUBS << ulog slots
  uint64_t* uval;   // (epoch << 32) | first admitted index, ~0 = none
  yrwi_hit* stack;  // 2 * q.k entries (double buffer)
};

struct EvJob {
  int32_t ev;       // index into the EvDev array
  int32_t local;
  const uint8_t* rows;
  int64_t n;
  // yrwi_event_order: the arrival only continues the event's ReferenceOrder
  // (min/max, max-distance fold, host counts) and every row's cardinal under the
  // state after it lands here; no doublecheck, flag counts or stack (the caller's
  // SearchEvent.addRWIs keeps those).  nullptr: a full addRWIs arrival.
  int64_t* scores;
};

// one workgroup per event: jobs [jb[b], jb[b+1]) of the same event, in arrival order; status[j] = 0 / YRWI_E_*
int launch_event_add(const EvDev* d_ev, const EvJob* d_jobs, const int32_t* d_jb, int32_t nblocks, int32_t* d_status,
                     void* stream);
// ---- TermSearch's urlselection (yrwi_query_desc.urlselection)
// url id of each of n url keys (0xFFFFFFFF: not in the url dictionary)
int launch_sel_lookup(const uint64_t* d_hi, const uint8_t* d_lo, int64_t n, const uint64_t* dkhi, const uint8_t* dklo,
                      int64_t nurls, uint32_t* d_uid, void* stream);
struct SelCount {
  ChainList L;           // an include or exclude list of the query
  const uint32_t* sel;   // the query's url ids (ascending)
  int64_t nsel;
  int64_t* out;          // |L restricted to the selection|
};
int launch_sel_count(const SelCount* d_jobs, int32_t njobs, void* stream);
// a single include list restricted to the selection, rows as they are stored
// (ReferenceContainerCache.get + the as-is single container, ReferenceContainer.java:355-370):
// one workgroup per query
struct SelPick {
  ChainList L;
  const uint64_t* feat;
  const uint8_t* rows;
  const uint32_t* sel;
  int64_t nsel;
  uint32_t* out_uid;
  uint64_t* out_feat;
  uint8_t* out_rows;
};
int launch_sel_pick(const SelPick* d_jobs, int32_t njobs, void* stream);
// ReferenceOrder.authority (ReferenceOrder.java:213-216) of n host keys (host36 + 1)
// against an event's accumulated host counts
int launch_event_authority(const EvDev* d_ev, const uint64_t* d_keys, int32_t n, int32_t* d_out, void* stream);
// (arrival epoch << 32 | row) of each url's admitted posting in the event's url set, ~0: absent
int launch_event_where(const EvDev* d_ev, const uint64_t* d_hi, const uint8_t* d_lo, int32_t n, uint64_t* d_out,
                       void* stream);
// seeds the url set with the doublecheck urls of the filter (epoch 0)
int launch_event_seed(const EvDev* d_ev, const uint64_t* d_hi, const uint8_t* d_lo, int64_t n, void* stream);

}  // namespace yrwi
