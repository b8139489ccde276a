/* yrwi.h -- C ABI of libyrwi, the MI355X-native YaCy RWI query engine.
 *
 * Drop-in boundary for YaCy's reverse-word-index query hot path.  Each entry
 * point names the Java interface it replaces (paths relative to
 * /root/reference/source/net/yacy).  INTEGRATION.md shows the JNI / Panama
 * binding a YaCy maintainer would add.
 *
 * Conventions:
 *   - int return codes: 0 = OK, < 0 = error (YRWI_E_*); message via yrwi_last_error();
 *   - "no result" is an empty result (n = 0), never an error -- as in
 *     ReferenceContainer.joinExcludeContainers (ReferenceContainer.java:318,322);
 *   - the caller owns every host buffer; the library owns device memory;
 *   - a context is bound to one GPU and is not thread-safe: one context per
 *     host thread, or serialise calls;
 *   - rows are YaCy's 40-byte WordReferenceRow layout (WordReferenceRow.java:49-72),
 *     i.e. the bytes of RowSet.chunkcache (RowCollection.java:68).
 */
#ifndef YRWI_H
#define YRWI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YRWI_ROW_BYTES 40
#define YRWI_HASH_BYTES 12
#define YRWI_MAX_TERMS 8          /* include or exclude terms per query */
#define YRWI_MAX_K 3000           /* WeakPriorityBlockingQueue bound, SearchEvent.java:118 */
#define YRWI_MAX_DISTANCE_ANY 2147483647 /* Integer.MAX_VALUE: unquoted query, yacysearch.java:643 */

enum {
  YRWI_OK = 0,
  YRWI_E_ARG = -1,           /* bad argument / capacity too small */
  YRWI_E_HASH = -2,          /* url or term hash not well-formed Base64 (Base64Order.java:96-106) */
  YRWI_E_UNSORTED = -3,      /* rows not strictly ascending by url hash (and sorted != 0) */
  YRWI_E_HIP = -4,           /* HIP runtime error */
  YRWI_E_NOMEM = -5,         /* device allocation failed (SpaceExceededException) */
  YRWI_E_RCCL = -6,          /* collective failed */
  YRWI_E_NULL_LANGUAGE = -7, /* language cell is 0x0000: the reference throws NPE in
                                ASCII.getBytes(null) (WordReferenceVars.java:315, ReferenceOrder.java:260) */
  YRWI_E_UNSUPPORTED = -8,
  YRWI_E_LIMIT = -9,         /* list longer than 53,687,091 rows (RowSet.java:90-92) */
  YRWI_E_CAPACITY = -10      /* search event tables full (max_postings given to yrwi_event_open too small) */
};

typedef struct yrwi_ctx yrwi_ctx;

/* RankingProfile public int coefficients, in the declaration order of
 * RankingProfile.java:81-88.  Defaults: yrwi_profile_default(). */
typedef struct yrwi_profile {
  int32_t coeff_domlength, coeff_date, coeff_wordsintitle, coeff_wordsintext, coeff_phrasesintext,
      coeff_llocal, coeff_lother, coeff_urllength, coeff_urlcomps, coeff_hitcount,
      coeff_posintext, coeff_posofphrase, coeff_posinphrase, coeff_authority, coeff_worddistance,
      coeff_appurl, coeff_app_dc_title, coeff_app_dc_creator, coeff_app_dc_subject,
      coeff_app_dc_description, coeff_appemph, coeff_catindexof, coeff_cathasimage,
      coeff_cathasaudio, coeff_cathasvideo, coeff_cathasapp, coeff_urlcompintoplist,
      coeff_descrcompintoplist, coeff_prefer, coeff_termfrequency, coeff_language, coeff_citation;
} yrwi_profile;

/* One ranked result: a ReverseElement of SearchEvent.rwiStack
 * (WeakPriorityBlockingQueue.java:400-426). */
typedef struct yrwi_hit {
  uint8_t urlhash[12];
  int32_t tiebreak; /* ByteArray.hashCode(urlhash) (ByteArray.java:80-84) */
  int64_t score;    /* ReferenceOrder.cardinal(WordReference) (ReferenceOrder.java:223-265) */
} yrwi_hit;

/* Per-query constraints that SearchEvent.addRWIs applies before a posting enters
 * rwiStack (SearchEvent.java:736-806), and the doubledom pull order of
 * pullOneRWI(skipDoubleDom) (:1297-1394).  Normalisation still covers the whole
 * joined container; these only decide which postings are ranked. */
typedef struct yrwi_filter {
  uint8_t constraint[4];        /* QueryParams.constraint as Bitfield bytes (bit j: byte j>>3, bit j&7) */
  int32_t has_constraint;       /* constraint != null; testFlags :2459-2474 */
  int32_t all_of_constraint;    /* QueryParams.allofconstraint */
  int32_t contentdom;           /* ContentDomain code: -1 ALL, 0 TEXT, 1 IMAGE, 2 AUDIO, 3 VIDEO, 4 APP */
  int32_t strict_contentdom;    /* QueryParams.isStrictContentDom(): test the doctype, not the flags */
  char language[8];             /* QueryModifier.language, NUL terminated; "" = any */
  uint8_t sitehash[6];          /* QueryModifier.sitehash: host hash = url-hash chars 6..11 */
  uint8_t alt_sitehash[6];      /* DigestURL.hosthash of the www./non-www. variant (:716-718) */
  int32_t has_sitehash, has_alt_sitehash;
  const uint8_t* siteexcludes;  /* nsiteexcludes * 6 bytes (QueryParams.siteexcludes); used without sitehash */
  int32_t nsiteexcludes;
  const uint8_t* urlhashes;     /* nurlhashes * 12 bytes already in SearchEvent.urlhashes (doublecheck) */
  int32_t nurlhashes;
  int32_t skip_double_dom;      /* results in pullOneRWI(true) order: new hosts first (stack bound 3000) */
  int32_t* flagcount;           /* out: SearchEvent.flagcount[32] over the postings past the doublecheck, or NULL */
} yrwi_filter;

/* A query: QueryGoal include/exclude word hashes (QueryGoal.java:229-240) plus
 * QueryParams.maxDistance, the ranking profile and the target language. */
typedef struct yrwi_query_desc {
  const uint8_t* incl;        /* nincl * 12 bytes (word hashes) */
  int32_t nincl;
  const uint8_t* excl;        /* nexcl * 12 bytes */
  int32_t nexcl;
  int32_t max_distance;       /* YRWI_MAX_DISTANCE_ANY or #terms-1 for quoted queries */
  int32_t k;                  /* results wanted (<= YRWI_MAX_K) */
  const yrwi_profile* profile;
  char language[8];           /* ReferenceOrder.language, NUL terminated (any length) */
  int64_t now_ms;             /* System.currentTimeMillis() of the request; 0 = now */
  const yrwi_filter* filter;  /* NULL: unconstrained query */
  /* TermSearch's urlselection (TermSearch.java:42-62 -> AbstractIndex.searchConjunction :96-128):
   * nurlselection url hashes (12 bytes each; NULL / 0: none).  Every include and exclude
   * container is restricted to these urls before the conjunction, as
   * ReferenceContainerCache.get(key, urlselection) does (ReferenceContainerCache.java:448-470):
   * J1, the J2 fold order and every J3 dispatch then see the restricted sizes.  (IndexCell.get,
   * YaCy's segment index, ignores the argument (IndexCell.java:353-386) and the local search
   * passes null (SearchEvent.java:619).)  A selection with two or more include terms runs as a
   * chained fold: more than four include terms, or a maxDistance filter (quoted query), with a
   * selection: YRWI_E_UNSUPPORTED. */
  const uint8_t* urlselection;
  int32_t nurlselection;
} yrwi_query_desc;

typedef struct yrwi_stats {
  int64_t postings_in;   /* sum of include + exclude list lengths */
  int64_t joined;        /* rows of the joined container (before exclusion) */
  int64_t bytes_alg;     /* algorithmic bytes B = sum K + 12 sum n_excl + 23 t m_out */
  int64_t bytes_join;    /* sum K over the merge-path join jobs (the k_join launches timed in t_join_ns), K as the
                            reference dispatches the step (J3) */
  int64_t t_join_ns;     /* device time of the k_join launches (HIP events on the context stream) */
  int64_t t_norm_ns, t_score_ns, t_total_ns;
  int32_t n_join_launches, n_enum_steps, n_test_steps;
  int32_t n_realloc;     /* device-wide allocation events (scratch or pinned staging growth) during the call */
  int64_t bytes_probe;   /* sum K over the probe-executed join jobs (timed in t_probe_ns), K as the reference
                            dispatches the step (J3) */
  int64_t t_probe_ns;    /* device time of the k_probe launches */
  int64_t bytes_compact; /* bytes k_compact moves: per joined row 12 B pair + url id read, the 32-B ranking
                            record of the accumulated side and 16 B of the joined side's (by-test steps: one
                            32-B record) read, 32-B record + url id written */
  int64_t t_compact_ns;  /* device time of the compaction launches (k_compact and / or k_compact_sum, which also
                            writes the normalisation pieces of the queries that need no other pass) */
  int64_t t_kernels_ns;  /* device time of all the batch's kernel launches (HIP events around every group of
                            back-to-back launches; host waits and collectives excluded) */
  /* SURVEY.md §8(d) bytes with no step credited for reads its kernel never makes: every join step
     (merge, probe, exclusion) is charged min(K, the bytes its kernel loads) -- merge tiles: 4-B url ids
     of both sides; url-id bitmap probe: the smaller side's 4-B ids + one 16-B bitmap word per id;
     range probe: the ids + the larger list's range or a 128-B leaf line per id, whichever is less.
     bytes_probe_loaded / _capped: the probe-executed include steps (k_probe); bytes_join_capped: the
     merge-executed include steps (k_join); bytes_alg_capped: the whole path (joins, exclusions and
     23 t m_out) */
  int64_t bytes_probe_loaded;
  int64_t bytes_probe_capped;
  int64_t bytes_features;    /* 23 t m_out: the ranking-feature bytes of the joined containers (k_compact's share) */
  int64_t bytes_join_capped;
  int64_t bytes_alg_capped;
  /* every k_probe dispatch of the call, include and exclusion steps alike (rocprofv3 counts them all):
     their number and device time (HIP events around each) */
  int64_t n_probe_dispatches;
  int64_t t_probe_all_ns;
  /* rank phase, per pass: the k_reduce launch (with k_piece_merge, which merges the compaction's pieces)
     and the k_score launches (k_shard_fin / k_score_full excluded: the populations rocprofv3 averages),
     HIP events around each; the bytes their kernels must read: k_reduce the 32-B ranking record of every
     joined row of the queries without pieces (+ its 1-B exclusion mark), k_score the same records of
     every query (an upper bound: chunks pruned by the per-query threshold read only words 2-3) */
  int64_t n_rank_passes;
  int64_t t_reduce_ns;
  int64_t t_scorek_ns;
  int64_t bytes_reduce;
  int64_t bytes_score;
  /* chained folds: the k_chain launches, their device time (HIP events around k_chain alone, the
     population rocprofv3 averages) and their SURVEY.md §8(d) bytes -- the later fold steps' K and the
     exclusions' 12 n_e, each charged min(K, the bytes k_chain loads for it) */
  int64_t n_chain_launches;
  int64_t t_chain_ns;
  int64_t bytes_chain;
} yrwi_stats;

/* ---- profile helpers (RankingProfile.java) ---- */
void yrwi_profile_default(yrwi_profile* p);                 /* RankingProfile(TEXT) :90-125 */
void yrwi_profile_all_zero(yrwi_profile* p);                /* allZero() :200-233 */
int yrwi_profile_parse(const char* prefix, const char* ext, yrwi_profile* out); /* :127-189 */

/* ---- context ---- */
int yrwi_open(int device, yrwi_ctx** out);
/* One shard of a URL-hash-range partitioned index (Distribution.java:153-158):
 * rank r of `world` (power of two) owns url hashes whose first character index
 * c satisfies c >> (6 - log2(world)) == r.  `nccl_id` is the 128-byte
 * ncclUniqueId from yrwi_get_unique_id() on rank 0, broadcast by the caller.
 * The shards merge their partial results over RCCL (Protocol.java:802 merges
 * peers' results).  The ranks of a node first post their devices' PCI bus ids
 * in the node's host mailbox: ranks that share one device (RCCL refuses a
 * duplicate GPU) run the device collectives host-staged through shared memory
 * instead, as does an id starting with "YRWI-HOSTSTAGE".  Ranks on distinct
 * devices use RCCL only: if ncclCommInitRank fails the call returns YRWI_E_RCCL
 * and yrwi_last_error(NULL) gives RCCL's error string.  yrwi_shard_info says
 * which transport a context runs on. */
int yrwi_open_shard(int device, int rank, int world, const uint8_t nccl_id[128], yrwi_ctx** out);
int yrwi_get_unique_id(uint8_t nccl_id[128]);
void yrwi_close(yrwi_ctx* ctx);
/* ctx's last error; NULL: why the calling thread's last yrwi_open / yrwi_open_shard failed */
const char* yrwi_last_error(yrwi_ctx* ctx);

enum {
  YRWI_TRANSPORT_NONE = 0,        /* not sharded (yrwi_open) */
  YRWI_TRANSPORT_RCCL = 1,        /* RCCL communicators (xGMI between the node's GPUs) */
  YRWI_TRANSPORT_HOSTSTAGED = 2,  /* ranks share one device: host shared memory (/dev/shm) */
  YRWI_TRANSPORT_LOOPBACK = 3     /* in-process test group */
};
typedef struct yrwi_transport_info {
  int32_t transport;       /* YRWI_TRANSPORT_* */
  int32_t rank, world;
  int32_t rccl_ranks;      /* ncclCommCount of lane 0's communicator (0: no communicator) */
  int32_t lanes;           /* lanes (batches in flight) */
  int32_t lanes_own_comm;  /* lanes with a communicator of their own (ncclCommSplit) */
  int32_t device_peers;    /* other ranks of the group on this rank's device (-1: not exchanged) */
  int32_t mailbox;         /* 1: list sizes summed through the node's host mailbox */
  char pci_bus_id[16];     /* this rank's device */
} yrwi_transport_info;
/* The transport of a (shard) context and its communicator's rank count:
 * Distribution.java:153-158 partitions, Protocol.java:802 merges over it. */
int yrwi_shard_info(yrwi_ctx* ctx, yrwi_transport_info* out);

/* ---- index (IndexCell.add / RowSet import; the lists are what
 *      Index.get(termHash) returns, IndexCell.java:353-386) ---- */
/* Stores (or replaces) the posting list of `term`.  rows40: n rows of 40 bytes.
 * sorted != 0 promises ascending unique url hashes (validated); sorted == 0
 * sorts (duplicate url hashes: the first occurrence wins, RowSet.mergeEnum). */
int yrwi_put_list(yrwi_ctx* ctx, const uint8_t term[12], const uint8_t* rows40, int64_t n, int sorted);
int yrwi_list_size(yrwi_ctx* ctx, const uint8_t term[12], int64_t* n);
/* Index.get(termHash) for callers off the query path (AbstractIndex.java:116,
 * IndexCell.java:353-386; e.g. TermSearch.inclusion() for the index abstracts,
 * SearchEvent.java:513-531): the 40-byte rows of `term`'s list on this context
 * (its url-hash shard when sharded), ascending by url hash.  *n = the list size
 * (0: no list); YRWI_E_ARG when cap < *n (nothing copied). */
int yrwi_get_list(yrwi_ctx* ctx, const uint8_t term[12], uint8_t* rows40, int64_t cap, int64_t* n);
/* Brings the url dictionary (url hash -> order-preserving 32-bit url id, the
 * join key in HBM) up to date now instead of at the next query.  The first
 * build sorts every key; later put_list / removal / load_heaps changes are
 * merged in incrementally (IndexCell.add, IndexCell.java:289): only the changed
 * lists' keys are sorted, keys new to the dictionary shift the ids after them
 * (the other lists' ids are remapped in one pass, not re-sorted), and keys of
 * removed postings stay until a full rebuild (when the changed lists hold over
 * a quarter of the postings, or removed ones over half; YRWI_DICT_FULL=1
 * forces it). */
int yrwi_build_url_ids(yrwi_ctx* ctx);
/* Diagnostic: brings the ids up to date, then *bad = postings whose id does not
 * name their url hash or does not ascend within its list, plus dictionary
 * entries out of order (0 when consistent); *nurls = dictionary size (may be NULL). */
int yrwi_check_url_ids(yrwi_ctx* ctx, int64_t* bad, int64_t* nurls);
int yrwi_index_stats(yrwi_ctx* ctx, int64_t* nterms, int64_t* npostings, int64_t* device_bytes);
/* Index maintenance counters (diagnostics and tests). */
typedef struct yrwi_index_info {
  int64_t full_rebuilds;        /* url dictionary built from every key */
  int64_t incremental_updates;  /* changed lists merged into an existing dictionary */
  int64_t repacks;              /* index memory compactions (dead bytes of replaced lists reclaimed) */
  int64_t index_bytes;          /* device bytes of the index arena (rows, keys, records, incremental ids) */
  int64_t index_bytes_used;     /* of which allocated so far (live + not yet reclaimed) */
  int64_t bitmap_lists;         /* lists with a url-id bitmap */
} yrwi_index_info;
int yrwi_index_info_get(yrwi_ctx* ctx, yrwi_index_info* info);
/* Device-wide allocation events of the process so far (scratch arena growth,
 * pinned staging growth: each one stalls every lane of the device while it
 * runs).  A caller counts them around a timed region without per-batch
 * statistics; steady-state batches make none. */
int64_t yrwi_realloc_events(void);
/* Sizes every lane's scratch arena and pinned staging to the largest any lane has
 * needed so far (one allocation each): call after a few representative batches,
 * and later batches of that workload make no device-wide allocation on any lane
 * (a lane otherwise grows on its own first large batch). */
int yrwi_settle_scratch(yrwi_ctx* ctx);
/* Diagnostic of the node's shared-memory size exchange (no GPU needed): rank
 * `rank` of `world` processes / threads sharing group id `id` runs `nparts`
 * batch parts of `ncalls` exchanges each, vectors of n values (rank + part +
 * call + i), and checks every sum.  0 when all sums are right; YRWI_E_RCCL on a
 * wrong sum or a peer that never arrives; 1 when the mailbox is unavailable.
 * n < 0 (vectors of -n values): the last rank's first part fails and aborts the
 * mailbox, as a failing batch part does; the others return YRWI_E_RCCL at once. */
int yrwi_hostx_selftest(const uint8_t id[128], int world, int rank, int64_t nparts, int32_t ncalls, int64_t n);

/* ---- YaCy on-disk index ---- */
/* Loads BLOB heap files of the RWI (records [int32 reclen][12-byte term hash]
 * [exported RowSet], HeapWriter.java:114-124, RowCollection.java:209-224) into
 * device memory.  Files are folded oldest first with RowSet.mergeEnum (the older
 * file's row wins on equal url hashes; ReferenceContainerArray.get :305-322);
 * lists already in the context act as the RAM cache and are merged below the
 * files (IndexCell.get :353-386).  A sharded context keeps only its url-hash
 * range.  With YRWI_LOAD_ORDER_BY_NAME the files are ordered by the
 * <prefix>.<yyyyMMddHHmmssSSS>.blob stamp and others are ignored
 * (ArrayStack.java:182-229); otherwise `paths` is taken as oldest first.
 * Malformed records are skipped as HeapReader does; a term whose RowSet export
 * is inconsistent (importRowSet's SpaceExceededException) keeps only its RAM
 * list, as does a term with malformed rows; both are counted in dropped_terms. */
#define YRWI_LOAD_ORDER_BY_NAME 1
typedef struct yrwi_load_stats {
  int64_t files, records, free_records, bad_keys;
  int64_t terms;          /* lists stored (replaced or new) */
  int64_t postings;       /* rows in those lists */
  int64_t dropped_terms;
} yrwi_load_stats;
int yrwi_load_heaps(yrwi_ctx* ctx, const char* const* paths, int32_t npaths, int32_t flags,
                    yrwi_load_stats* st);

/* ---- query hot path ---- */
/* TermSearch + joinExcludeContainers + normalizeWith + cardinal + rwiStack top-k
 * (SearchEvent.RWIProcess.run :612-631 -> addRWIs :673-836), canonical
 * deterministic semantics.  out: k hits, best first. */
int yrwi_query(yrwi_ctx* ctx, const yrwi_query_desc* q, yrwi_hit* out, int32_t* nout, yrwi_stats* st);
/* nq independent queries in one device pass (throughput mode).
 * out: nq * kmax hits (row q at out + q*kmax), nout[q] = hits of query q. */
int yrwi_query_batch(yrwi_ctx* ctx, const yrwi_query_desc* q, int32_t nq, int32_t kmax,
                     yrwi_hit* out, int32_t* nout, yrwi_stats* st);

/* Asynchronous batches (throughput mode: SearchEvent runs many RWIProcess
 * feeders concurrently, SearchEvent.java:612-631).  submit returns at once with
 * a ticket; the batch runs on one of the context's lanes (own HIP stream and
 * host thread) while the caller prepares the next one.  q, the profiles it
 * points to, out, nout and st must stay valid until yrwi_query_batch_wait(ticket)
 * returns; every ticket must be waited for exactly once.  Lists must not be
 * changed while batches are in flight (put_list waits for them).  Sharded
 * contexts: every rank submits the same batches in the same order (the batches'
 * device collectives are enqueued in submission order). */
int yrwi_query_batch_submit(yrwi_ctx* ctx, const yrwi_query_desc* q, int32_t nq, int32_t kmax,
                            yrwi_hit* out, int32_t* nout, yrwi_stats* st, int64_t* ticket);
int yrwi_query_batch_wait(yrwi_ctx* ctx, int64_t ticket);

/* Pinned host memory for result buffers: hits written into such a buffer come
 * straight from the GPU (no staging copy).  Free with yrwi_host_free. */
int yrwi_host_alloc(yrwi_ctx* ctx, size_t bytes, void** p);
int yrwi_host_free(yrwi_ctx* ctx, void* p);

/* ---- Solr node stack ---- */
/* The fields of a URIMetadataNode that ReferenceOrder.cardinal(URIMetadataNode)
 * reads (ReferenceOrder.java:267-296); the caller extracts them from the Solr
 * document (URIMetadataNode.java:238-504). */
typedef struct yrwi_node {
  uint8_t urlhash[12];    /* t.hash() */
  int32_t virtual_age;    /* t.virtualAge() = MicroDate.microDateDays(moddate) */
  int32_t wordsintitle;   /* t.wordsintitle() */
  int32_t wordcount;      /* t.wordCount() */
  int32_t llocal, lother; /* t.llocal(), t.lother() */
  uint8_t flags[4];       /* t.flags() Bitfield bytes */
  int32_t host_count;     /* ReferenceOrder.doms.get(t.hosthash()) (authority) */
  char language[8];       /* t.language(), NUL terminated; "" = null */
} yrwi_node;
/* scores[i] = cardinal(nodes[i]) under `prof` and the ReferenceOrder language;
 * maxdomcount is ReferenceOrder.maxdomcount (authority divisor 1 + maxdomcount). */
int yrwi_score_nodes(yrwi_ctx* ctx, const yrwi_node* nodes, int64_t n, const yrwi_profile* prof,
                     const char* language, int32_t maxdomcount, int64_t* scores);

/* ---- search events: local + remote containers merged per arrival ---- */
/* A SearchEvent's RWI side (SearchEvent.java:673-836): containers arrive one
 * after another -- the local joined container from RWIProcess.run (:612-631) and
 * each remote peer's result container from Protocol.remoteSearchProcess
 * (Protocol.java:670-830, addRWIs(container, false, ...) at :802).  Every
 * arrival continues the event's ReferenceOrder (min/max, max-distance fold,
 * host counts), is settled over itself and then scored; entries already on the
 * stack keep their arrival-time scores.  The doublecheck set (SearchEvent.
 * urlhashes), the flag counts and the rwiStack (bound k) persist in device
 * memory.  Rows are WordReferenceRow bytes in the container's order (a remote
 * container is in the order the peer's results arrived). */
typedef struct yrwi_event yrwi_event;
/* k: stack bound (<= YRWI_MAX_K; the results kept); filter: constraints, its
 * urlhashes seed the doublecheck set (NULL: unconstrained; its flagcount and
 * skip_double_dom are not used -- see yrwi_event_result, yrwi_event_pull); max_postings: the
 * most postings the event will receive (sizes the url and host tables). */
int yrwi_event_open(yrwi_ctx* ctx, const yrwi_profile* prof, const char* language, int64_t now_ms, int32_t k,
                    const yrwi_filter* filter, int64_t max_postings, yrwi_event** out);
/* An event for yrwi_event_order / yrwi_event_authority only (GpuReferenceOrder: the
 * ReferenceOrder of a SearchEvent whose addRWIs stays in Java): no url set and no
 * stack, the host table first sized for max_hosts distinct hosts (authority
 * profiles) and grown by yrwi_event_order before a container could fill it
 * (ReferenceOrder.doms is unbounded, ReferenceOrder.java:176-198), device memory
 * reused from closed order-only events.
 * The event entry points serialise on the context (callers on several threads). */
int yrwi_event_open_order(yrwi_ctx* ctx, const yrwi_profile* prof, const char* language, int64_t now_ms,
                          int64_t max_hosts, yrwi_event** out);
typedef struct yrwi_arrival {
  yrwi_event* ev;
  const uint8_t* rows40;  /* n rows of 40 bytes */
  int64_t n;
  int32_t local;          /* addRWIs(local): statistics only */
  int32_t rc;             /* out: 0 or YRWI_E_* (HASH, NULL_LANGUAGE, CAPACITY) for this arrival */
} yrwi_arrival;
/* Applies arrivals in array order (per event); arrivals of different events run
 * in parallel, one workgroup per event.  Returns the first nonzero rc. */
int yrwi_event_add(yrwi_ctx* ctx, yrwi_arrival* arr, int32_t narr);
/* ReferenceOrder.normalizeWith(container, local) + cardinal of each of its rows
 * for a drop-in ReferenceOrder whose SearchEvent.addRWIs stays in Java
 * (ReferenceOrder.java:70-79,163-265; GpuReferenceOrder): the container continues
 * the event's ReferenceOrder exactly as an arrival does -- min/max and the
 * max-distance fold accumulate over every container given so far, the host counts
 * (doms, maxdomcount) too -- and scores[i] = cardinal(row i) under the state after
 * this container (settled over it).  The event's doublecheck set,
 * flag counts and stack are not touched (addRWIs keeps its own).  Do not mix
 * with yrwi_event_add on one event. */
int yrwi_event_order(yrwi_ctx* ctx, yrwi_event* ev, const uint8_t* rows40, int64_t n, int32_t local,
                     int64_t* scores);
/* ReferenceOrder.authority(hostHash) (ReferenceOrder.java:213-216) against the
 * event's accumulated host counts: out[i] = (doms(h_i) << 8) / (1 + maxdomcount),
 * h_i the 6-character host hash at hosts6 + 6 i (url-hash chars 6..11).  The
 * counts exist when the event's profile has coeff_authority > 12 (else 0). */
int yrwi_event_authority(yrwi_ctx* ctx, yrwi_event* ev, const uint8_t* hosts6, int32_t n, int32_t* out);
typedef struct yrwi_event_info {
  int32_t flagcount[32];        /* SearchEvent.flagcount */
  int64_t postings_in;          /* rows received */
  int64_t admitted_local;       /* local_rwi_available */
  int64_t admitted_remote;      /* remote_rwi_available */
  int64_t remote_arrivals;      /* remote_rwi_peerCount */
  int32_t maxdomcount;          /* ReferenceOrder.maxdomcount (authority profiles only) */
  int32_t max_distance;         /* max.distance() of the fold (min.distance() is 0) */
  int32_t err;                  /* YRWI_E_CAPACITY once the event's tables overflowed */
  int32_t stack_size;
} yrwi_event_info;
/* Where each url entered the event's doublecheck set (SearchEvent.urlhashes,
 * :736-805: the first posting of the url that passed the constraints):
 * arrival[i] = its yrwi_event_add arrival (1 = the event's first), row[i] = its row
 * in that arrival's rows; arrival 0 = seeded by the filter's urlhashes; -1 = not in
 * the set.  A caller that keeps the arrivals' rows (GpuRWIStack) turns a pulled hit
 * back into its posting. */
int yrwi_event_source(yrwi_ctx* ctx, yrwi_event* ev, const uint8_t* urls12, int32_t n, int32_t* arrival,
                      int32_t* row);
/* The stack in rwiStack order (best first), up to maxn entries. */
int yrwi_event_result(yrwi_ctx* ctx, yrwi_event* ev, yrwi_hit* out, int32_t maxn, int32_t* nout,
                      yrwi_event_info* info);
/* SearchEvent.pullOneRWI(skip_double_dom) (SearchEvent.java:1297-1394) repeated
 * up to maxn times, stopping where it returns null: each pull polls the event's
 * rwiStack (the entry leaves it, so later arrivals fill the bound again); with
 * skip_double_dom, an entry whose host was already returned goes to that host's
 * doubleDomCache queue, and after 10 such polls (or an empty stack) the best head
 * of those queues is returned (a host whose queue empties leaves the cache).  The
 * cache persists across calls and arrivals.  Equal heads of different hosts go
 * by ReverseElement order, then the earliest queued (the reference walks a
 * ConcurrentHashMap).  Every url is taken to have metadata (the fulltext lookup
 * at :1309,1327,1392 is not on the RWI path). */
int yrwi_event_pull(yrwi_ctx* ctx, yrwi_event* ev, int32_t skip_double_dom, yrwi_hit* out, int32_t maxn,
                    int32_t* nout);
void yrwi_event_close(yrwi_ctx* ctx, yrwi_event* ev);

/* ---- index abstracts and the secondary search ---- */
/* AbstractIndex.searchConjunction + WordReferenceFactory.compressIndex for each
 * term (htroot/yacy/search.java:264-281, SearchEvent.java:505-531;
 * WordReferenceFactory.java:75-117 without its time limit): "{host:u6u6...,host:...}"
 * with hosts in String order and url prefixes in container order, minus the urls
 * of exclude_term's list (NULL: none).  Abstract i is out[offsets[i],
 * offsets[i+1]); *nout = nterms, or 0 when a term has no list (searchConjunction
 * returns no containers then). */
int yrwi_index_abstracts(yrwi_ctx* ctx, const uint8_t* terms, int32_t nterms, const uint8_t* exclude_term,
                         char* out, int64_t cap, int64_t* offsets, int32_t* nout);
/* One index abstract received from a peer (Protocol.java:576-596). */
typedef struct yrwi_abstract {
  uint8_t word[12];
  uint8_t peer[12];
  const char* text;
  int64_t len;
} yrwi_abstract;
/* A secondary search request (SecondarySearchSuperviser.prepareSecondarySearch
 * :117-196): the peer, the words to ask it for (bit i = words_out[i]) and its urls
 * (plan_urls[url_off .. url_off + url_n), 12 bytes each, String order). */
typedef struct yrwi_peer_request {
  uint8_t peer[12];
  uint32_t words;
  int64_t url_off, url_n;
} yrwi_peer_request;
/* decompressIndex of every abstract (in arrival order), addAbstract, the
 * joinConstructive of the words and the requests for the peers other than
 * mypeer and `checked` (SecondarySearchSuperviser.java:43-196, WordReferenceFactory.
 * java:125-155, SetTools.java:76-116).  Nothing is planned unless the abstracts
 * cover exactly nwords_query words.  Outputs: the join (njoin urls in String
 * order with their peer), words_out (the words in String order, <= 32), the
 * requests in peer order.  A text that is not a compressIndex abstract fails with
 * YRWI_E_ARG (the reference would read past its buffer); one without braces is
 * an empty abstract. */
int yrwi_secondary_search(yrwi_ctx* ctx, const yrwi_abstract* abs, int32_t nabs, int32_t nwords_query,
                          const uint8_t mypeer[12], const uint8_t* checked, int32_t nchecked,
                          uint8_t* join_urls, uint8_t* join_peers, int64_t cap, int64_t* njoin,
                          yrwi_peer_request* plan, int32_t plan_cap, int32_t* nplan, uint8_t* plan_urls,
                          uint8_t* words_out, int32_t* nwords);

/* ---- finer-grained drop-ins mirroring the Java split ---- */
/* == ReferenceContainer.joinExcludeContainers via TermSearch (ReferenceContainer.java:310,
 *    TermSearch.java:42-70): writes the joined container's rows (sorted) to rows_out. */
int yrwi_join_exclude(yrwi_ctx* ctx, const uint8_t* incl, int32_t nincl, const uint8_t* excl,
                      int32_t nexcl, int32_t max_distance, int64_t now_ms, uint8_t* rows_out,
                      int64_t cap_rows, int64_t* m);
/* == ReferenceOrder.normalizeWith + cardinal (ReferenceOrder.java:70,223) on one
 *    container (rows sorted by url hash), with settled min/max: score_out[i] =
 *    cardinal(row i). */
/* TermSearch(index, include, exclude, urlselection, ...).joined() for one query
 * descriptor (the urlselection of yrwi_query_desc honoured; k, profile, language
 * and filter unused): the joined and excluded container's rows, as
 * yrwi_join_exclude writes them. */
int yrwi_term_search(yrwi_ctx* ctx, const yrwi_query_desc* q, uint8_t* rows40_out, int64_t cap_rows, int64_t* m);
int yrwi_normalize_score(yrwi_ctx* ctx, const uint8_t* rows40, int64_t m, const yrwi_profile* prof,
                         const char* language, int64_t now_ms, int64_t* score_out);

#ifdef __cplusplus
}
#endif
#endif /* YRWI_H */
