/* yrwi_jni.c -- JNI glue between net.yacy.kelondro.rwi.GpuRWI and libyrwi.
 * UNVERIFIED (no JDK / jni.h in this image); see INTEGRATION.md.
 * Build on a JDK host:
 *   cc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *      yrwi_jni.c -L../../yacy_search_server_amd -lyrwi -o libyrwi_jni.so */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include "yrwi.h"

/* A Java byte[] of at least `need` bytes copied into native memory (no critical
 * region around library calls that synchronise with the GPU: GC stays free);
 * NULL (IllegalArgumentException pending) when the array is shorter, or on OOM. */
static uint8_t* copy_in(JNIEnv* env, jbyteArray a, int64_t need) {
  if (a == NULL || need < 0 || (int64_t)(*env)->GetArrayLength(env, a) < need) {
    jclass ex = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (ex) (*env)->ThrowNew(env, ex, "array shorter than n rows / hosts");
    return NULL;
  }
  uint8_t* b = (uint8_t*)malloc((size_t)(need > 0 ? need : 1));
  if (b && need > 0) (*env)->GetByteArrayRegion(env, a, 0, (jsize)need, (jbyte*)b);
  return b;
}

static void to_profile(JNIEnv* env, jintArray a, yrwi_profile* p) {
  if (a == NULL) { yrwi_profile_default(p); return; }
  (*env)->GetIntArrayRegion(env, a, 0, 32, (jint*)p);
}

JNIEXPORT jlong JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_open(JNIEnv* env, jclass c, jint dev) {
  yrwi_ctx* ctx = NULL;
  return yrwi_open(dev, &ctx) == 0 ? (jlong)(intptr_t)ctx : 0;
}

JNIEXPORT void JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_close(JNIEnv* env, jclass c, jlong ctx) {
  yrwi_close((yrwi_ctx*)(intptr_t)ctx);
}

JNIEXPORT jint JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_putList(JNIEnv* env, jclass c, jlong ctx, jbyteArray term,
                                                                jbyteArray rows, jint n, jint sorted) {
  jbyte t[12];
  (*env)->GetByteArrayRegion(env, term, 0, 12, t);
  uint8_t* p = copy_in(env, rows, (int64_t)n * 40);
  if (!p) return YRWI_E_ARG;
  int rc = yrwi_put_list((yrwi_ctx*)(intptr_t)ctx, (const uint8_t*)t, p, n, sorted);
  free(p);
  return rc;
}

JNIEXPORT jbyteArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_joinExclude(JNIEnv* env, jclass c, jlong ctx,
                                                                          jbyteArray incl, jint nincl, jbyteArray excl,
                                                                          jint nexcl, jint maxd, jlong now) {
  yrwi_ctx* x = (yrwi_ctx*)(intptr_t)ctx;
  jbyte* ib = (*env)->GetByteArrayElements(env, incl, NULL);
  jbyte* eb = (*env)->GetByteArrayElements(env, excl, NULL);
  int64_t cap = 0, n;
  for (int i = 0; i < nincl; i++) {
    if (yrwi_list_size(x, (const uint8_t*)ib + 12 * i, &n) == 0 && n > cap) cap = n;
  }
  uint8_t* out = (uint8_t*)malloc((size_t)(cap > 0 ? cap : 1) * 40);
  int64_t m = 0;
  int rc = yrwi_join_exclude(x, (const uint8_t*)ib, nincl, (const uint8_t*)eb, nexcl, maxd, now, out, cap, &m);
  (*env)->ReleaseByteArrayElements(env, incl, ib, JNI_ABORT);
  (*env)->ReleaseByteArrayElements(env, excl, eb, JNI_ABORT);
  jbyteArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewByteArray(env, (jsize)(m * 40));
    (*env)->SetByteArrayRegion(env, res, 0, (jsize)(m * 40), (const jbyte*)out);
  }
  free(out);
  return res;  /* null on error (caller: yrwi_last_error) */
}

/* TermSearch(..., urlselection, ...).joined(): every list restricted to the url
 * selection (n * 12 bytes) before the conjunction (yrwi_term_search) */
JNIEXPORT jbyteArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_termSearch(JNIEnv* env, jclass c, jlong ctx,
                                                                         jbyteArray incl, jint nincl, jbyteArray excl,
                                                                         jint nexcl, jbyteArray sel, jint nsel,
                                                                         jint maxd, jlong now) {
  yrwi_ctx* x = (yrwi_ctx*)(intptr_t)ctx;
  jbyte* ib = (*env)->GetByteArrayElements(env, incl, NULL);
  jbyte* eb = (*env)->GetByteArrayElements(env, excl, NULL);
  jbyte* sb = sel ? (*env)->GetByteArrayElements(env, sel, NULL) : NULL;
  int64_t cap = 0, n;
  for (int i = 0; i < nincl; i++) {
    if (yrwi_list_size(x, (const uint8_t*)ib + 12 * i, &n) == 0 && n > cap) cap = n;
  }
  uint8_t* out = (uint8_t*)malloc((size_t)(cap > 0 ? cap : 1) * 40);
  yrwi_query_desc q;
  memset(&q, 0, sizeof(q));
  q.incl = (const uint8_t*)ib; q.nincl = nincl;
  q.excl = (const uint8_t*)eb; q.nexcl = nexcl;
  q.max_distance = maxd; q.k = 1; q.now_ms = now;
  q.urlselection = (const uint8_t*)sb; q.nurlselection = sb ? nsel : 0;
  int64_t m = 0;
  int rc = out ? yrwi_term_search(x, &q, out, cap, &m) : YRWI_E_NOMEM;
  (*env)->ReleaseByteArrayElements(env, incl, ib, JNI_ABORT);
  (*env)->ReleaseByteArrayElements(env, excl, eb, JNI_ABORT);
  if (sb) (*env)->ReleaseByteArrayElements(env, sel, sb, JNI_ABORT);
  jbyteArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewByteArray(env, (jsize)(m * 40));
    (*env)->SetByteArrayRegion(env, res, 0, (jsize)(m * 40), (const jbyte*)out);
  }
  free(out);
  return res;
}

/* joinExclude into a direct ByteBuffer the caller owns and reuses (no JNI array copy
 * of the joined container): returns m (rows written, 40 bytes each) or the (negative)
 * error code -- YRWI_E_ARG when the container holds more rows than capacity / 40. */
JNIEXPORT jlong JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_joinExcludeInto(JNIEnv* env, jclass c, jlong ctx,
                                                                         jbyteArray incl, jint nincl,
                                                                         jbyteArray excl, jint nexcl, jint maxd,
                                                                         jlong now, jobject out) {
  uint8_t* dst = (uint8_t*)(*env)->GetDirectBufferAddress(env, out);
  const jlong capb = (*env)->GetDirectBufferCapacity(env, out);
  if (dst == NULL || capb < 0) return YRWI_E_ARG;
  jbyte* ib = (*env)->GetByteArrayElements(env, incl, NULL);
  jbyte* eb = (*env)->GetByteArrayElements(env, excl, NULL);
  int64_t m = 0;
  int rc = yrwi_join_exclude((yrwi_ctx*)(intptr_t)ctx, (const uint8_t*)ib, nincl, (const uint8_t*)eb, nexcl, maxd, now,
                             dst, capb / 40, &m);
  (*env)->ReleaseByteArrayElements(env, incl, ib, JNI_ABORT);
  (*env)->ReleaseByteArrayElements(env, excl, eb, JNI_ABORT);
  return rc == 0 ? (jlong)m : (jlong)rc;
}

/* yrwi_stats -> long[]: postings_in, joined, bytes_alg, bytes_join, t_join_ns, t_norm_ns,
 * t_score_ns, t_total_ns, n_join_launches, n_enum_steps, n_test_steps, n_realloc,
 * bytes_probe, t_probe_ns, bytes_compact, t_compact_ns, t_kernels_ns (17 values) */
#define YRWI_JNI_NSTATS 17
static void stats_out(JNIEnv* env, jlongArray a, const yrwi_stats* st) {
  if (a == NULL) return;
  const jlong v[YRWI_JNI_NSTATS] = {st->postings_in, st->joined, st->bytes_alg, st->bytes_join, st->t_join_ns,
                                    st->t_norm_ns, st->t_score_ns, st->t_total_ns, st->n_join_launches,
                                    st->n_enum_steps, st->n_test_steps, st->n_realloc, st->bytes_probe,
                                    st->t_probe_ns, st->bytes_compact, st->t_compact_ns, st->t_kernels_ns};
  jsize n = (*env)->GetArrayLength(env, a);
  (*env)->SetLongArrayRegion(env, a, 0, n < YRWI_JNI_NSTATS ? n : YRWI_JNI_NSTATS, v);
}

JNIEXPORT jlongArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_normalizeScore(JNIEnv* env, jclass c, jlong ctx,
                                                                             jbyteArray rows, jint m, jintArray prof,
                                                                             jstring lang, jlong now) {
  yrwi_profile p;
  to_profile(env, prof, &p);
  const char* l = (*env)->GetStringUTFChars(env, lang, NULL);
  uint8_t* r = copy_in(env, rows, (int64_t)m * 40);
  if (!r) { (*env)->ReleaseStringUTFChars(env, lang, l); return NULL; }
  jlong* sc = (jlong*)malloc(sizeof(jlong) * (size_t)(m > 0 ? m : 1));
  int rc = sc ? yrwi_normalize_score((yrwi_ctx*)(intptr_t)ctx, r, m, &p, l, now, (int64_t*)sc) : YRWI_E_NOMEM;
  free(r);
  (*env)->ReleaseStringUTFChars(env, lang, l);
  jlongArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewLongArray(env, m);
    (*env)->SetLongArrayRegion(env, res, 0, m, sc);
  }
  free(sc);
  return res;
}

JNIEXPORT jbyteArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_query(JNIEnv* env, jclass c, jlong ctx,
                                                                    jbyteArray incl, jint nincl, jbyteArray excl,
                                                                    jint nexcl, jint maxd, jint k, jintArray prof,
                                                                    jstring lang, jlong now, jlongArray stats) {
  yrwi_profile p;
  to_profile(env, prof, &p);
  yrwi_query_desc q;
  memset(&q, 0, sizeof(q));
  jbyte* ib = (*env)->GetByteArrayElements(env, incl, NULL);
  jbyte* eb = (*env)->GetByteArrayElements(env, excl, NULL);
  const char* l = (*env)->GetStringUTFChars(env, lang, NULL);
  q.incl = (const uint8_t*)ib; q.nincl = nincl;
  q.excl = (const uint8_t*)eb; q.nexcl = nexcl;
  q.max_distance = maxd; q.k = k; q.profile = &p; q.now_ms = now;
  strncpy(q.language, l, sizeof(q.language) - 1);
  yrwi_hit* hits = (yrwi_hit*)malloc(sizeof(yrwi_hit) * (size_t)(k > 0 ? k : 1));
  int32_t n = 0;
  yrwi_stats st;
  memset(&st, 0, sizeof(st));
  int rc = yrwi_query((yrwi_ctx*)(intptr_t)ctx, &q, hits, &n, stats ? &st : NULL);
  (*env)->ReleaseByteArrayElements(env, incl, ib, JNI_ABORT);
  (*env)->ReleaseByteArrayElements(env, excl, eb, JNI_ABORT);
  (*env)->ReleaseStringUTFChars(env, lang, l);
  jbyteArray res = NULL;
  if (rc == 0) {
    stats_out(env, stats, &st);
    res = (*env)->NewByteArray(env, (jsize)(n * (jint)sizeof(yrwi_hit)));
    (*env)->SetByteArrayRegion(env, res, 0, (jsize)(n * (jint)sizeof(yrwi_hit)), (const jbyte*)hits);
  }
  free(hits);
  return res;
}

/* IndexCell's BLOB files (ReferenceContainerArray): yrwi_load_heaps; returns the
 * stats as long[7] {files, records, free_records, bad_keys, terms, postings, dropped_terms}. */
JNIEXPORT jlongArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_loadHeaps(JNIEnv* env, jclass c, jlong ctx,
                                                                        jobjectArray paths, jint byName) {
  const jsize n = (*env)->GetArrayLength(env, paths);
  const char** p = (const char**)calloc((size_t)(n > 0 ? n : 1), sizeof(char*));
  jstring* js = (jstring*)calloc((size_t)(n > 0 ? n : 1), sizeof(jstring));
  for (jsize i = 0; i < n; i++) {
    js[i] = (jstring)(*env)->GetObjectArrayElement(env, paths, i);
    p[i] = (*env)->GetStringUTFChars(env, js[i], NULL);
  }
  yrwi_load_stats st;
  int rc = yrwi_load_heaps((yrwi_ctx*)(intptr_t)ctx, p, n, byName ? YRWI_LOAD_ORDER_BY_NAME : 0, &st);
  for (jsize i = 0; i < n; i++) (*env)->ReleaseStringUTFChars(env, js[i], p[i]);
  free(p);
  free(js);
  if (rc != 0) return NULL;
  jlong v[7] = {st.files, st.records, st.free_records, st.bad_keys, st.terms, st.postings, st.dropped_terms};
  jlongArray res = (*env)->NewLongArray(env, 7);
  (*env)->SetLongArrayRegion(env, res, 0, 7, v);
  return res;
}

/* SearchEvent.addRWIs constraints + pullOneRWI(skipDoubleDom): query with a yrwi_filter.
 * constraint: 4 Bitfield bytes or null; site / altSite: 6-byte host hashes or null;
 * siteExcludes: n*6 bytes; urlHashes: n*12 bytes; flagCount: int[32] out or null. */
JNIEXPORT jbyteArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_queryFiltered(
    JNIEnv* env, jclass c, jlong ctx, jbyteArray incl, jint nincl, jbyteArray excl, jint nexcl, jint maxd, jint k,
    jintArray prof, jstring lang, jlong now, jbyteArray constraint, jboolean allOf, jint contentdom,
    jboolean strictDom, jstring modLang, jbyteArray site, jbyteArray altSite, jbyteArray siteExcludes,
    jbyteArray urlHashes, jboolean skipDoubleDom, jintArray flagCount) {
  yrwi_profile p;
  to_profile(env, prof, &p);
  yrwi_filter f;
  memset(&f, 0, sizeof(f));
  if (constraint) { (*env)->GetByteArrayRegion(env, constraint, 0, 4, (jbyte*)f.constraint); f.has_constraint = 1; }
  f.all_of_constraint = allOf;
  f.contentdom = contentdom;
  f.strict_contentdom = strictDom;
  if (modLang) {
    const char* ml = (*env)->GetStringUTFChars(env, modLang, NULL);
    strncpy(f.language, ml, sizeof(f.language) - 1);
    (*env)->ReleaseStringUTFChars(env, modLang, ml);
  }
  if (site) { (*env)->GetByteArrayRegion(env, site, 0, 6, (jbyte*)f.sitehash); f.has_sitehash = 1; }
  if (altSite) { (*env)->GetByteArrayRegion(env, altSite, 0, 6, (jbyte*)f.alt_sitehash); f.has_alt_sitehash = 1; }
  jbyte* sx = siteExcludes ? (*env)->GetByteArrayElements(env, siteExcludes, NULL) : NULL;
  jbyte* uh = urlHashes ? (*env)->GetByteArrayElements(env, urlHashes, NULL) : NULL;
  f.siteexcludes = (const uint8_t*)sx;
  f.nsiteexcludes = sx ? (*env)->GetArrayLength(env, siteExcludes) / 6 : 0;
  f.urlhashes = (const uint8_t*)uh;
  f.nurlhashes = uh ? (*env)->GetArrayLength(env, urlHashes) / 12 : 0;
  f.skip_double_dom = skipDoubleDom;
  int32_t fc[32];
  f.flagcount = flagCount ? fc : NULL;
  yrwi_query_desc q;
  memset(&q, 0, sizeof(q));
  jbyte* ib = (*env)->GetByteArrayElements(env, incl, NULL);
  jbyte* eb = (*env)->GetByteArrayElements(env, excl, NULL);
  const char* l = (*env)->GetStringUTFChars(env, lang, NULL);
  q.incl = (const uint8_t*)ib; q.nincl = nincl;
  q.excl = (const uint8_t*)eb; q.nexcl = nexcl;
  q.max_distance = maxd; q.k = k; q.profile = &p; q.now_ms = now; q.filter = &f;
  strncpy(q.language, l, sizeof(q.language) - 1);
  yrwi_hit* hits = (yrwi_hit*)malloc(sizeof(yrwi_hit) * (size_t)(k > 0 ? k : 1));
  int32_t n = 0;
  int rc = yrwi_query((yrwi_ctx*)(intptr_t)ctx, &q, hits, &n, NULL);
  (*env)->ReleaseByteArrayElements(env, incl, ib, JNI_ABORT);
  (*env)->ReleaseByteArrayElements(env, excl, eb, JNI_ABORT);
  if (sx) (*env)->ReleaseByteArrayElements(env, siteExcludes, sx, JNI_ABORT);
  if (uh) (*env)->ReleaseByteArrayElements(env, urlHashes, uh, JNI_ABORT);
  (*env)->ReleaseStringUTFChars(env, lang, l);
  jbyteArray res = NULL;
  if (rc == 0) {
    if (flagCount) (*env)->SetIntArrayRegion(env, flagCount, 0, 32, (const jint*)fc);
    res = (*env)->NewByteArray(env, (jsize)(n * (jint)sizeof(yrwi_hit)));
    (*env)->SetByteArrayRegion(env, res, 0, (jsize)(n * (jint)sizeof(yrwi_hit)), (const jbyte*)hits);
  }
  free(hits);
  return res;
}

/* ---- search events (SearchEvent.addRWIs per arrival) ---- */
JNIEXPORT jlong JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventOpen(JNIEnv* env, jclass c, jlong ctx, jintArray prof,
                                                                   jstring lang, jlong now, jint k, jlong maxPostings) {
  yrwi_profile p;
  to_profile(env, prof, &p);
  const char* l = (*env)->GetStringUTFChars(env, lang, NULL);
  yrwi_event* ev = NULL;
  int rc = yrwi_event_open((yrwi_ctx*)(intptr_t)ctx, &p, l, now, k, NULL, maxPostings, &ev);
  (*env)->ReleaseStringUTFChars(env, lang, l);
  return rc == 0 ? (jlong)(intptr_t)ev : 0;
}

/* GpuRWIStack's event: url set, rwiStack and doubleDomCache under the addRWIs constraints
 * (the same filter fields as queryFiltered; urlHashes seed the doublecheck set) */
JNIEXPORT jlong JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventOpenFiltered(
    JNIEnv* env, jclass c, jlong ctx, jintArray prof, jstring lang, jlong now, jint k, jlong maxPostings,
    jbyteArray constraint, jboolean allOf, jint contentdom, jboolean strictDom, jstring modLang, jbyteArray site,
    jbyteArray altSite, jbyteArray siteExcludes, jbyteArray urlHashes) {
  yrwi_profile p;
  to_profile(env, prof, &p);
  yrwi_filter f;
  memset(&f, 0, sizeof(f));
  if (constraint) { (*env)->GetByteArrayRegion(env, constraint, 0, 4, (jbyte*)f.constraint); f.has_constraint = 1; }
  f.all_of_constraint = allOf;
  f.contentdom = contentdom;
  f.strict_contentdom = strictDom;
  if (modLang) {
    const char* ml = (*env)->GetStringUTFChars(env, modLang, NULL);
    strncpy(f.language, ml, sizeof(f.language) - 1);
    (*env)->ReleaseStringUTFChars(env, modLang, ml);
  }
  if (site) { (*env)->GetByteArrayRegion(env, site, 0, 6, (jbyte*)f.sitehash); f.has_sitehash = 1; }
  if (altSite) { (*env)->GetByteArrayRegion(env, altSite, 0, 6, (jbyte*)f.alt_sitehash); f.has_alt_sitehash = 1; }
  const jsize nsx = siteExcludes ? (*env)->GetArrayLength(env, siteExcludes) / 6 : 0;
  const jsize nuh = urlHashes ? (*env)->GetArrayLength(env, urlHashes) / 12 : 0;
  uint8_t* sx = nsx ? copy_in(env, siteExcludes, (int64_t)nsx * 6) : NULL;
  uint8_t* uh = nuh ? copy_in(env, urlHashes, (int64_t)nuh * 12) : NULL;
  f.siteexcludes = sx;
  f.nsiteexcludes = sx ? nsx : 0;
  f.urlhashes = uh;
  f.nurlhashes = uh ? nuh : 0;
  const char* l = (*env)->GetStringUTFChars(env, lang, NULL);
  yrwi_event* ev = NULL;
  int rc = yrwi_event_open((yrwi_ctx*)(intptr_t)ctx, &p, l, now, k, &f, maxPostings, &ev);
  (*env)->ReleaseStringUTFChars(env, lang, l);
  free(sx);
  free(uh);
  return rc == 0 ? (jlong)(intptr_t)ev : 0;
}

/* (arrival, row) of the admitted posting of each of n url hashes (yrwi_event_source): int[2n] */
JNIEXPORT jintArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventSource(JNIEnv* env, jclass c, jlong ctx, jlong ev,
                                                                         jbyteArray urls, jint n) {
  uint8_t* u = copy_in(env, urls, (int64_t)n * 12);
  if (!u) return NULL;
  int32_t* a = (int32_t*)malloc(sizeof(int32_t) * 2 * (size_t)(n > 0 ? n : 1));
  int rc = a ? yrwi_event_source((yrwi_ctx*)(intptr_t)ctx, (yrwi_event*)(intptr_t)ev, u, n, a, a + (n > 0 ? n : 1))
             : YRWI_E_NOMEM;
  free(u);
  jintArray res = NULL;
  if (rc == 0) {
    jint* v = (jint*)malloc(sizeof(jint) * 2 * (size_t)(n > 0 ? n : 1));
    for (jint i = 0; v && i < n; i++) { v[2 * i] = a[i]; v[2 * i + 1] = a[(n > 0 ? n : 1) + i]; }
    res = (*env)->NewIntArray(env, 2 * n);
    if (v) (*env)->SetIntArrayRegion(env, res, 0, 2 * n, v);
    free(v);
  }
  free(a);
  return res;
}

/* SearchEvent.flagcount of an event (yrwi_event_result's info, no hits copied) */
JNIEXPORT jintArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventFlagCount(JNIEnv* env, jclass c, jlong ctx,
                                                                            jlong ev) {
  yrwi_event_info info;
  int32_t n = 0;
  if (yrwi_event_result((yrwi_ctx*)(intptr_t)ctx, (yrwi_event*)(intptr_t)ev, NULL, 0, &n, &info) != 0) return NULL;
  jintArray res = (*env)->NewIntArray(env, 32);
  (*env)->SetIntArrayRegion(env, res, 0, 32, (const jint*)info.flagcount);
  return res;
}

/* GpuReferenceOrder's event: the ReferenceOrder state and host table only (yrwi_event_open_order) */
JNIEXPORT jlong JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventOpenOrder(JNIEnv* env, jclass c, jlong ctx,
                                                                        jintArray prof, jstring lang, jlong now,
                                                                        jlong maxHosts) {
  yrwi_profile p;
  to_profile(env, prof, &p);
  const char* l = (*env)->GetStringUTFChars(env, lang, NULL);
  yrwi_event* ev = NULL;
  int rc = yrwi_event_open_order((yrwi_ctx*)(intptr_t)ctx, &p, l, now, maxHosts, &ev);
  (*env)->ReleaseStringUTFChars(env, lang, l);
  return rc == 0 ? (jlong)(intptr_t)ev : 0;
}

/* addRWIs(container, local): rows = RowSet.chunkcache bytes of the container in its order */
JNIEXPORT jint JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventAdd(JNIEnv* env, jclass c, jlong ctx, jlong ev,
                                                                 jbyteArray rows, jint n, jboolean local) {
  yrwi_arrival a;
  memset(&a, 0, sizeof(a));
  uint8_t* p = copy_in(env, rows, (int64_t)n * 40);
  if (!p) return YRWI_E_ARG;
  a.ev = (yrwi_event*)(intptr_t)ev;
  a.rows40 = p;
  a.n = n;
  a.local = local ? 1 : 0;
  int rc = yrwi_event_add((yrwi_ctx*)(intptr_t)ctx, &a, 1);
  free(p);
  return rc;
}

/* ReferenceOrder.normalizeWith + cardinal continuing the event's ReferenceOrder
 * (yrwi_event_order): one score per row of the container, in its order */
JNIEXPORT jlongArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventOrder(JNIEnv* env, jclass c, jlong ctx, jlong ev,
                                                                         jbyteArray rows, jint n, jboolean local) {
  /* yrwi_event_order drains the context and synchronises with the GPU: the rows are
   * copied out of the Java heap first (no GC-blocking critical region around it) */
  uint8_t* p = copy_in(env, rows, (int64_t)n * 40);
  if (!p) return NULL;
  jlong* sc = (jlong*)malloc(sizeof(jlong) * (size_t)(n > 0 ? n : 1));
  if (!sc) { free(p); return NULL; }
  int rc = yrwi_event_order((yrwi_ctx*)(intptr_t)ctx, (yrwi_event*)(intptr_t)ev, p, n, local ? 1 : 0, (int64_t*)sc);
  free(p);
  jlongArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewLongArray(env, n);
    (*env)->SetLongArrayRegion(env, res, 0, n, sc);
  }
  free(sc);
  return res;
}

/* ReferenceOrder.authority of n 6-byte host hashes against the event's host counts */
JNIEXPORT jintArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventAuthority(JNIEnv* env, jclass c, jlong ctx,
                                                                            jlong ev, jbyteArray hosts6, jint n) {
  uint8_t* h = copy_in(env, hosts6, (int64_t)n * 6);
  if (!h) return NULL;
  jint* out = (jint*)malloc(sizeof(jint) * (size_t)(n > 0 ? n : 1));
  int rc = out ? yrwi_event_authority((yrwi_ctx*)(intptr_t)ctx, (yrwi_event*)(intptr_t)ev, h, n, (int32_t*)out)
               : YRWI_E_NOMEM;
  free(h);
  jintArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewIntArray(env, n);
    (*env)->SetIntArrayRegion(env, res, 0, n, out);
  }
  free(out);
  return res;
}

/* rwiStack contents (yrwi_hit records) */
JNIEXPORT jbyteArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventResult(JNIEnv* env, jclass c, jlong ctx, jlong ev,
                                                                          jint maxn) {
  yrwi_hit* hits = (yrwi_hit*)malloc(sizeof(yrwi_hit) * (size_t)(maxn > 0 ? maxn : 1));
  int32_t n = 0;
  int rc = yrwi_event_result((yrwi_ctx*)(intptr_t)ctx, (yrwi_event*)(intptr_t)ev, hits, maxn, &n, NULL);
  jbyteArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewByteArray(env, (jsize)(n * (jint)sizeof(yrwi_hit)));
    (*env)->SetByteArrayRegion(env, res, 0, (jsize)(n * (jint)sizeof(yrwi_hit)), (const jbyte*)hits);
  }
  free(hits);
  return res;
}

/* pullOneRWI(skipDoubleDom) up to maxn times (SearchEvent.java:1297-1394): the
 * entries leave the event's rwiStack; yrwi_hit records in pull order */
JNIEXPORT jbyteArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventPull(JNIEnv* env, jclass c, jlong ctx, jlong ev,
                                                                        jboolean skipDoubleDom, jint maxn) {
  yrwi_hit* hits = (yrwi_hit*)malloc(sizeof(yrwi_hit) * (size_t)(maxn > 0 ? maxn : 1));
  int32_t n = 0;
  int rc = yrwi_event_pull((yrwi_ctx*)(intptr_t)ctx, (yrwi_event*)(intptr_t)ev, skipDoubleDom ? 1 : 0, hits, maxn, &n);
  jbyteArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewByteArray(env, (jsize)(n * (jint)sizeof(yrwi_hit)));
    (*env)->SetByteArrayRegion(env, res, 0, (jsize)(n * (jint)sizeof(yrwi_hit)), (const jbyte*)hits);
  }
  free(hits);
  return res;
}

JNIEXPORT void JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_eventClose(JNIEnv* env, jclass c, jlong ctx, jlong ev) {
  yrwi_event_close((yrwi_ctx*)(intptr_t)ctx, (yrwi_event*)(intptr_t)ev);
}

/* ---- index abstracts: compressIndex per term (searchConjunction), one String each ---- */
JNIEXPORT jobjectArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_indexAbstracts(JNIEnv* env, jclass c, jlong ctx,
                                                                               jbyteArray terms, jint nterms,
                                                                               jlong cap) {
  jbyte* tb = (*env)->GetByteArrayElements(env, terms, NULL);
  char* out = (char*)malloc((size_t)(cap > 0 ? cap : 1) + 1);
  int64_t* off = (int64_t*)calloc((size_t)nterms + 1, sizeof(int64_t));
  int32_t nout = 0;
  int rc = yrwi_index_abstracts((yrwi_ctx*)(intptr_t)ctx, (const uint8_t*)tb, nterms, NULL, out, cap, off, &nout);
  (*env)->ReleaseByteArrayElements(env, terms, tb, JNI_ABORT);
  jobjectArray res = NULL;
  if (rc == 0) {  /* abstract i = bytes [off[i], off[i+1]) (ASCII); none when a term has no list */
    res = (*env)->NewObjectArray(env, nout, (*env)->FindClass(env, "java/lang/String"), NULL);
    for (int32_t i = 0; i < nout; i++) {
      const char save = out[off[i + 1]];
      out[off[i + 1]] = 0;
      jstring s = (*env)->NewStringUTF(env, out + off[i]);
      out[off[i + 1]] = save;
      (*env)->SetObjectArrayElement(env, res, i, s);
      (*env)->DeleteLocalRef(env, s);
    }
  }
  free(out);
  free(off);
  return res;
}

/* ---- Index.size / Index.get of the GPU index (J1 sizes, TermSearch.inclusion) ---- */
JNIEXPORT jlongArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_listSizes(JNIEnv* env, jclass c, jlong ctx,
                                                                        jbyteArray terms, jint nterms) {
  jbyte* tb = (*env)->GetByteArrayElements(env, terms, NULL);
  jlong* v = (jlong*)calloc((size_t)(nterms > 0 ? nterms : 1), sizeof(jlong));
  int rc = 0;
  for (jint i = 0; i < nterms && rc == 0; i++) {
    int64_t n = 0;
    rc = yrwi_list_size((yrwi_ctx*)(intptr_t)ctx, (const uint8_t*)tb + 12 * i, &n);
    v[i] = n;
  }
  (*env)->ReleaseByteArrayElements(env, terms, tb, JNI_ABORT);
  jlongArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewLongArray(env, nterms);
    (*env)->SetLongArrayRegion(env, res, 0, nterms, v);
  }
  free(v);
  return res;
}

JNIEXPORT jbyteArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_getList(JNIEnv* env, jclass c, jlong ctx,
                                                                      jbyteArray term) {
  yrwi_ctx* x = (yrwi_ctx*)(intptr_t)ctx;
  jbyte t[12];
  (*env)->GetByteArrayRegion(env, term, 0, 12, t);
  int64_t n = 0, m = 0;
  if (yrwi_list_size(x, (const uint8_t*)t, &n) != 0) return NULL;
  jbyteArray res = (*env)->NewByteArray(env, (jsize)(n * 40));
  if (n == 0) return res;
  /* the device copy lands in a native buffer first: no GC-blocking critical region
   * around the copy and its stream synchronisation.  yrwi_get_list drains the
   * context's batches; it must not run concurrently with yrwi_put_list (one
   * context per host thread, include/yrwi.h). */
  uint8_t* buf = (uint8_t*)malloc((size_t)n * 40);
  if (!buf) return NULL;
  int rc = yrwi_get_list(x, (const uint8_t*)t, buf, n, &m);
  if (rc == 0 && m == n) (*env)->SetByteArrayRegion(env, res, 0, (jsize)(n * 40), (const jbyte*)buf);
  free(buf);
  return rc == 0 && m == n ? res : NULL;
}

/* ---- Solr node stack: cardinal(URIMetadataNode); nodes = packed yrwi_node records ---- */
JNIEXPORT jlongArray JNICALL Java_net_yacy_kelondro_rwi_GpuRWI_scoreNodes(JNIEnv* env, jclass c, jlong ctx,
                                                                         jbyteArray nodes, jint n, jintArray prof,
                                                                         jstring lang, jint maxdomcount) {
  yrwi_profile p;
  to_profile(env, prof, &p);
  const char* l = (*env)->GetStringUTFChars(env, lang, NULL);
  jbyte* nb = (*env)->GetByteArrayElements(env, nodes, NULL);
  jlong* sc = (jlong*)malloc(sizeof(jlong) * (size_t)(n > 0 ? n : 1));
  int rc = yrwi_score_nodes((yrwi_ctx*)(intptr_t)ctx, (const yrwi_node*)nb, n, &p, l, maxdomcount, (int64_t*)sc);
  (*env)->ReleaseByteArrayElements(env, nodes, nb, JNI_ABORT);
  (*env)->ReleaseStringUTFChars(env, lang, l);
  jlongArray res = NULL;
  if (rc == 0) {
    res = (*env)->NewLongArray(env, n);
    (*env)->SetLongArrayRegion(env, res, 0, n, sc);
  }
  free(sc);
  return res;
}
