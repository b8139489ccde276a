// GpuRWI.java -- JNI binding of libyrwi (include/yrwi.h) for YaCy.
//
// UNVERIFIED: this image has no JDK (no javac, no jni.h), so this file and
// java/jni/yrwi_jni.c are shipped as the binding a YaCy maintainer would add;
// they have not been compiled here.  See INTEGRATION.md.
//
// Drop-in points (paths relative to source/net/yacy):
//   kelondro/rwi/TermSearch.java:42-70         -> GpuRWI.listSizes(...) + joinExclude(...) / termSearch(...) (GpuTermSearch)
//   kelondro/rwi/AbstractIndex.java:116        -> GpuRWI.getList(...) (TermSearch.inclusion, on demand)
//   kelondro/rwi/ReferenceContainer.java:310   -> GpuRWI.joinExclude(...)
//   search/ranking/ReferenceOrder.java:70,223  -> GpuRWI.eventOrder(...) (GpuReferenceOrder: one event per SearchEvent)
//   search/query/SearchEvent.java:612-631      -> GpuRWI.query(...) (whole local RWI path)
//   search/query/SearchEvent.java:736-806,1297 -> GpuRWI.queryFiltered(...) (constraints, doubledom)
//   kelondro/rwi/IndexCell.java:353-386        -> GpuRWI.loadHeaps(...) (BLOB heaps into HBM)
//
// Java level: 1.8, YaCy's own (build.properties javacSource/javacTarget, pom.xml
// maven.compiler.source/target).  No API newer than Java 8 is used here or in the
// other drop-ins (tests/test_java_sequence.py scans java/ for them).
package net.yacy.kelondro.rwi;

import java.lang.ref.PhantomReference;
import java.lang.ref.Reference;
import java.lang.ref.ReferenceQueue;
import java.util.ArrayList;
import java.util.Collections;
import java.util.Set;
import java.util.concurrent.ConcurrentHashMap;

public final class GpuRWI implements AutoCloseable {

    // A libyrwi context is not thread-safe (include/yrwi.h): every call on it is
    // synchronized on this object.  YaCy reaches one GpuRWI from the search threads,
    // the remote-peer (Protocol) threads and the result workers (authority()).

    static { System.loadLibrary("yrwi_jni"); }  // links libyrwi.so

    private long ctx;  // yrwi_ctx*

    /**
     * The release of one search event (GpuReferenceOrder, GpuRWIStack), Java 8 style:
     * a phantom reference to the object that owns the event.  The owner's close()
     * calls release(); an owner dropped without close() is released by this
     * context's reaper thread once the collector has enqueued the reference
     * (java.lang.ref.Cleaner does the same from Java 9 on, which YaCy's 1.8 build
     * does not have).  release() runs at most once.
     */
    public static final class EventHandle extends PhantomReference<Object> {
        private final GpuRWI gpu;
        private long event;

        EventHandle(final Object owner, final GpuRWI gpu, final long event, final ReferenceQueue<Object> q) {
            super(owner, q);
            this.gpu = gpu;
            this.event = event;
        }

        public void release() {
            final long e;
            synchronized (this) { e = this.event; this.event = 0; }
            if (e == 0) return;
            this.gpu.handles.remove(this);
            this.gpu.eventClose(e);
        }
    }

    private final ReferenceQueue<Object> unreachable = new ReferenceQueue<Object>();
    // the handles must stay strongly reachable until released, or they are collected themselves
    private final Set<EventHandle> handles = Collections.newSetFromMap(new ConcurrentHashMap<EventHandle, Boolean>());
    private final Thread reaper;

    public GpuRWI(final int device) {
        this.ctx = open(device);
        if (this.ctx == 0) throw new IllegalStateException("yrwi_open failed");
        final ReferenceQueue<Object> q = this.unreachable;
        this.reaper = new Thread(new Runnable() {
            @Override
            public void run() {
                while (true) {
                    final Reference<?> r;
                    try { r = q.remove(); } catch (final InterruptedException e) { return; }
                    if (r instanceof EventHandle) ((EventHandle) r).release();
                }
            }
        }, "GpuRWI event reaper");
        this.reaper.setDaemon(true);
        this.reaper.start();
    }

    /** Registers `event` for release when `owner` becomes unreachable (or at close()). */
    public EventHandle track(final Object owner, final long event) {
        final EventHandle h = new EventHandle(owner, this, event, this.unreachable);
        this.handles.add(h);
        return h;
    }

    /** IndexCell.add for a whole container: the RowSet chunkcache bytes (n * 40, sorted). */
    public synchronized void putList(final byte[] termHash, final byte[] chunkcache, final int n) {
        check(putList(this.ctx, termHash, chunkcache, n, 1));
    }

    /** Index.size(termHash) of each term on the GPU index (yrwi_list_size; 0: no list). */
    public synchronized long[] listSizes(final byte[][] terms) {
        return listSizes(this.ctx, flatten(terms), terms.length);
    }

    /** Index.get(termHash) off the query path (yrwi_get_list): the list's sorted rows (n * 40 bytes). */
    public synchronized byte[] getList(final byte[] term) {
        final byte[] rows = getList(this.ctx, term);
        if (rows == null) throw new IllegalStateException("yrwi_get_list failed");
        return rows;
    }

    /** TermSearch + joinExcludeContainers: returns the joined container's rows (m * 40 bytes). */
    public synchronized byte[] joinExclude(final byte[][] include, final byte[][] exclude, final int maxDistance,
                              final long nowMillis) {
        return joinExclude(this.ctx, flatten(include), include.length, flatten(exclude), exclude.length,
                           maxDistance, nowMillis);
    }

    /** TermSearch(..., urlselection, ...).joined(): every include and exclude list restricted
     *  to the url selection (url hashes) before the conjunction, as
     *  ReferenceContainerCache.get(key, urlselection) restricts it (yrwi_term_search). */
    public synchronized byte[] termSearch(final byte[][] include, final byte[][] exclude, final byte[][] urlselection,
                             final int maxDistance, final long nowMillis) {
        final byte[] rows = termSearch(this.ctx, flatten(include), include.length, flatten(exclude), exclude.length,
                                       urlselection == null ? null : flatten(urlselection),
                                       urlselection == null ? 0 : urlselection.length, maxDistance, nowMillis);
        if (rows == null) throw new IllegalStateException("yrwi_term_search failed");
        return rows;
    }

    /** joinExclude into a caller-owned direct buffer (ByteBuffer.allocateDirect, reused
     *  across queries): no copy of the joined container through a Java array.  Returns
     *  the number of 40-byte rows written; throws when the container does not fit. */
    public synchronized long joinExcludeInto(final byte[][] include, final byte[][] exclude, final int maxDistance,
                                final long nowMillis, final java.nio.ByteBuffer out) {
        final long m = joinExcludeInto(this.ctx, flatten(include), include.length, flatten(exclude), exclude.length,
                                       maxDistance, nowMillis, out);
        if (m < 0) check((int) m);
        return m;
    }

    /** ReferenceOrder.normalizeWith + cardinal with settled min/max: one score per row. */
    public synchronized long[] normalizeScore(final byte[] rows, final int m, final int[] profile32, final String language,
                                 final long nowMillis) {
        return normalizeScore(this.ctx, rows, m, profile32, language, nowMillis);
    }

    /** SearchEvent local RWI path: top-k (urlhash, cardinal) of one query. Output: k * 24 bytes
     *  (12-byte url hash, int32 ByteArray.hashCode, int64 score), little endian. */
    public synchronized byte[] query(final byte[][] include, final byte[][] exclude, final int maxDistance, final int k,
                        final int[] profile32, final String language, final long nowMillis) {
        return query(this.ctx, flatten(include), include.length, flatten(exclude), exclude.length, maxDistance, k,
                     profile32, language, nowMillis, null);
    }

    /** query(...) with the call's yrwi_stats (17 longs, order in yrwi_jni.c stats_out):
     *  postings in, joined rows, algorithmic bytes, per-phase device times, launches. */
    public synchronized byte[] query(final byte[][] include, final byte[][] exclude, final int maxDistance, final int k,
                        final int[] profile32, final String language, final long nowMillis, final long[] stats) {
        return query(this.ctx, flatten(include), include.length, flatten(exclude), exclude.length, maxDistance, k,
                     profile32, language, nowMillis, stats);
    }

    /** IndexCell's BLOB heaps (text.index.*.blob) into the GPU index; lists already
     *  present act as the RAM cache.  Returns {files, records, free, badKeys, terms,
     *  postings, droppedTerms}. */
    public synchronized long[] loadHeaps(final String[] heapFiles, final boolean orderByFileName) {
        return loadHeaps(this.ctx, heapFiles, orderByFileName ? 1 : 0);
    }

    /** query(...) under SearchEvent.addRWIs constraints (SearchEvent.java:736-806) and,
     *  with skipDoubleDom, in pullOneRWI order (:1297-1394).  flagCount (int[32] or null)
     *  receives SearchEvent.flagcount. */
    public synchronized byte[] queryFiltered(final byte[][] include, final byte[][] exclude, final int maxDistance, final int k,
                                final int[] profile32, final String language, final long nowMillis,
                                final byte[] constraint, final boolean allOfConstraint, final int contentdom,
                                final boolean strictContentDom, final String modifierLanguage, final byte[] sitehash,
                                final byte[] altSitehash, final byte[][] siteexcludes, final byte[][] urlhashes,
                                final boolean skipDoubleDom, final int[] flagCount) {
        return queryFiltered(this.ctx, flatten(include), include.length, flatten(exclude), exclude.length,
                             maxDistance, k, profile32, language, nowMillis, constraint, allOfConstraint, contentdom,
                             strictContentDom, modifierLanguage, sitehash, altSitehash, flattenN(siteexcludes, 6),
                             flattenN(urlhashes, 12), skipDoubleDom, flagCount);
    }

    /** A SearchEvent's rwiStack on the GPU: open once per event, then addRWIs for the
     *  local container and every remote peer's container (Protocol.java:802); the
     *  result is the stack in rwiStack order (24-byte records as query()). */
    public synchronized long eventOpen(final int[] profile32, final String language, final long nowMillis, final int k,
                          final long maxPostings) {
        return eventOpen(this.ctx, profile32, language, nowMillis, k, maxPostings);
    }

    /** SearchEvent.addRWIs constraints of one event (SearchEvent.java:736-806), the
     *  fields of QueryParams queryFiltered takes; null arrays: no such constraint. */
    public static final class EventFilter {
        public byte[] constraint;          // Bitfield bytes (4) or null
        public boolean allOfConstraint;
        public int contentdom = -1;        // ContentDomain code, -1: ALL
        public boolean strictContentDom;
        public String modifierLanguage;    // QueryModifier.language or null
        public byte[] sitehash, altSitehash;  // 6-byte host hashes or null
        public byte[][] siteexcludes;      // 6-byte host hashes or null
        public byte[][] urlhashes;         // url hashes already in SearchEvent.urlhashes (doublecheck) or null
    }

    /** A full search event (url set, rwiStack, doubleDomCache) under constraints: GpuRWIStack. */
    public synchronized long eventOpenFiltered(final int[] profile32, final String language, final long nowMillis,
                                               final int k, final long maxPostings, final EventFilter f) {
        if (f == null) return eventOpen(this.ctx, profile32, language, nowMillis, k, maxPostings);
        return eventOpenFiltered(this.ctx, profile32, language, nowMillis, k, maxPostings, f.constraint,
                                 f.allOfConstraint, f.contentdom, f.strictContentDom, f.modifierLanguage, f.sitehash,
                                 f.altSitehash, flattenN(f.siteexcludes, 6), flattenN(f.urlhashes, 12));
    }

    /** (arrival, row) pairs of the postings the event's doublecheck admitted for n url
     *  hashes (12 bytes each): arrival 1 = the first addRWIs, 0 = seeded, -1 = absent. */
    public synchronized int[] eventSource(final long event, final byte[] urls, final int n) {
        final int[] s = eventSource(this.ctx, event, urls, n);
        if (s == null) throw new IllegalStateException("yrwi_event_source failed");
        return s;
    }

    /** SearchEvent.flagcount of an event (yrwi_event_result's info). */
    public synchronized int[] eventFlagCount(final long event) {
        final int[] fc = eventFlagCount(this.ctx, event);
        if (fc == null) throw new IllegalStateException("yrwi_event_result failed");
        return fc;
    }

    /** An event holding only a SearchEvent's ReferenceOrder (yrwi_event_open_order):
     *  eventOrder / eventAuthority only, the host table sized for maxHosts hosts; device
     *  memory comes from closed order-only events (no device-wide allocation per event). */
    public synchronized long eventOpenOrder(final int[] profile32, final String language, final long nowMillis,
                                            final long maxHosts) {
        return eventOpenOrder(this.ctx, profile32, language, nowMillis, maxHosts);
    }

    public synchronized void addRWIs(final long event, final byte[] containerRows, final int n, final boolean local) {
        check(eventAdd(this.ctx, event, containerRows, n, local));
    }

    /** ReferenceOrder.normalizeWith(container, local) + cardinal of every row, continuing
     *  the event's ReferenceOrder (yrwi_event_order): min/max, the max-distance fold and
     *  the host counts accumulate over every container given to the event; the scores
     *  are under the state after this one.  The event's stack is not touched. */
    public synchronized long[] eventOrder(final long event, final byte[] containerRows, final int n, final boolean local) {
        final long[] sc = eventOrder(this.ctx, event, containerRows, n, local);
        if (sc == null) throw new IllegalStateException("yrwi_event_order failed");
        return sc;
    }

    /** ReferenceOrder.authority(hostHash) against the event's accumulated host counts. */
    public synchronized int eventAuthority(final long event, final byte[] hostHash6) {
        final int[] a = eventAuthority(this.ctx, event, hostHash6, 1);
        if (a == null) throw new IllegalStateException("yrwi_event_authority failed");
        return a[0];
    }

    /** eventAuthority for n host hashes at once (6 bytes each, concatenated): one call. */
    public synchronized int[] eventAuthorities(final long event, final byte[] hostHashes6, final int n) {
        final int[] a = eventAuthority(this.ctx, event, hostHashes6, n);
        if (a == null) throw new IllegalStateException("yrwi_event_authority failed");
        return a;
    }

    public synchronized byte[] eventResult(final long event, final int maxn) {
        return eventResult(this.ctx, event, maxn);
    }

    /** SearchEvent.pullOneRWI(skipDoubleDom) up to maxn times (SearchEvent.java:1297-1394):
     *  yrwi_hit records (12-byte url hash, int hashCode, long score) in pull order;
     *  the entries leave the event's rwiStack, the doubleDomCache stays with the event. */
    public synchronized byte[] pullRWI(final long event, final boolean skipDoubleDom, final int maxn) {
        return eventPull(this.ctx, event, skipDoubleDom, maxn);
    }

    public synchronized void eventClose(final long event) {
        if (this.ctx != 0) eventClose(this.ctx, event);  // after close() the context freed it
    }

    /** WordReferenceFactory.compressIndex of each include word's list (search.java:264-281):
     *  one "{...}" per word; empty when a word has no list (searchConjunction is empty). */
    public synchronized String[] indexAbstracts(final byte[][] words, final long capacity) {
        return indexAbstracts(this.ctx, flatten(words), words.length, capacity);
    }

    /** ReferenceOrder.cardinal(URIMetadataNode) of packed yrwi_node records (60 bytes each). */
    public synchronized long[] scoreNodes(final byte[] nodes, final int n, final int[] profile32, final String language,
                             final int maxdomcount) {
        return scoreNodes(this.ctx, nodes, n, profile32, language, maxdomcount);
    }

    @Override
    public synchronized void close() {
        if (this.ctx == 0) return;
        this.reaper.interrupt();
        for (final EventHandle h : new ArrayList<EventHandle>(this.handles)) h.release();  // events before the context
        close(this.ctx);
        this.ctx = 0;
    }

    /** RankingProfile public coefficients in declaration order (RankingProfile.java:81-88). */
    public static int[] profile32(final net.yacy.search.ranking.RankingProfile p) {
        return new int[] {
            p.coeff_domlength, p.coeff_date, p.coeff_wordsintitle, p.coeff_wordsintext, p.coeff_phrasesintext,
            p.coeff_llocal, p.coeff_lother, p.coeff_urllength, p.coeff_urlcomps, p.coeff_hitcount,
            p.coeff_posintext, p.coeff_posofphrase, p.coeff_posinphrase, p.coeff_authority, p.coeff_worddistance,
            p.coeff_appurl, p.coeff_app_dc_title, p.coeff_app_dc_creator, p.coeff_app_dc_subject,
            p.coeff_app_dc_description, p.coeff_appemph, p.coeff_catindexof, p.coeff_cathasimage,
            p.coeff_cathasaudio, p.coeff_cathasvideo, p.coeff_cathasapp, p.coeff_urlcompintoplist,
            p.coeff_descrcompintoplist, p.coeff_prefer, p.coeff_termfrequency, p.coeff_language, p.coeff_citation};
    }

    private static byte[] flatten(final byte[][] hashes) {
        final byte[] b = new byte[12 * hashes.length];
        for (int i = 0; i < hashes.length; i++) System.arraycopy(hashes[i], 0, b, 12 * i, 12);
        return b;
    }

    private static byte[] flattenN(final byte[][] hashes, final int w) {
        if (hashes == null) return null;
        final byte[] b = new byte[w * hashes.length];
        for (int i = 0; i < hashes.length; i++) System.arraycopy(hashes[i], 0, b, w * i, w);
        return b;
    }

    private static void check(final int rc) {
        if (rc != 0) throw new IllegalStateException("libyrwi error " + rc);
    }

    private static native long open(int device);
    private static native void close(long ctx);
    private static native int putList(long ctx, byte[] term, byte[] rows, int n, int sorted);
    private static native byte[] joinExclude(long ctx, byte[] incl, int nincl, byte[] excl, int nexcl,
                                             int maxDistance, long nowMillis);
    private static native long[] normalizeScore(long ctx, byte[] rows, int m, int[] profile32, String language,
                                                long nowMillis);
    private static native byte[] termSearch(long ctx, byte[] incl, int nincl, byte[] excl, int nexcl, byte[] sel,
                                            int nsel, int maxDistance, long nowMillis);
    private static native long joinExcludeInto(long ctx, byte[] incl, int nincl, byte[] excl, int nexcl,
                                               int maxDistance, long nowMillis, java.nio.ByteBuffer out);
    private static native byte[] query(long ctx, byte[] incl, int nincl, byte[] excl, int nexcl, int maxDistance,
                                       int k, int[] profile32, String language, long nowMillis, long[] stats);
    private static native long[] loadHeaps(long ctx, String[] paths, int byName);
    private static native byte[] queryFiltered(long ctx, byte[] incl, int nincl, byte[] excl, int nexcl,
                                               int maxDistance, int k, int[] profile32, String language,
                                               long nowMillis, byte[] constraint, boolean allOf, int contentdom,
                                               boolean strictDom, String modifierLanguage, byte[] site,
                                               byte[] altSite, byte[] siteExcludes, byte[] urlHashes,
                                               boolean skipDoubleDom, int[] flagCount);
    private static native long eventOpen(long ctx, int[] profile32, String language, long nowMillis, int k,
                                         long maxPostings);
    private static native long eventOpenFiltered(long ctx, int[] profile32, String language, long nowMillis, int k,
                                                 long maxPostings, byte[] constraint, boolean allOf, int contentdom,
                                                 boolean strictDom, String modifierLanguage, byte[] site,
                                                 byte[] altSite, byte[] siteExcludes, byte[] urlHashes);
    private static native int[] eventFlagCount(long ctx, long event);
    private static native int[] eventSource(long ctx, long event, byte[] urls, int n);
    private static native long eventOpenOrder(long ctx, int[] profile32, String language, long nowMillis,
                                              long maxHosts);
    private static native int eventAdd(long ctx, long event, byte[] rows, int n, boolean local);
    private static native byte[] eventResult(long ctx, long event, int maxn);
    private static native long[] eventOrder(long ctx, long event, byte[] rows, int n, boolean local);
    private static native int[] eventAuthority(long ctx, long event, byte[] hosts6, int n);
    private static native byte[] eventPull(long ctx, long event, boolean skipDoubleDom, int maxn);
    private static native void eventClose(long ctx, long event);
    private static native String[] indexAbstracts(long ctx, byte[] words, int nwords, long capacity);
    private static native long[] listSizes(long ctx, byte[] terms, int nterms);
    private static native byte[] getList(long ctx, byte[] term);
    private static native long[] scoreNodes(long ctx, byte[] nodes, int n, int[] profile32, String language,
                                            int maxdomcount);
}
