// GpuRWIStack.java -- a SearchEvent's RWI side on the GPU: addRWIs + rwiStack +
// pullOneRWI (SURVEY.md §8f row 3; UNVERIFIED: no JDK in this image).
//
// Replaces (paths relative to source/net/yacy):
//   search/query/SearchEvent.java:673-836    addRWIs: normalizeWith, the per-posting
//                                            doublecheck (RowHandleSet), testFlags /
//                                            contentdom / language / site constraints,
//                                            flag counts and the rwiStack put
//                                            -> yrwi_event_add (one kernel per arrival)
//   search/query/SearchEvent.java:1297-1394  pullOneRWI(skipDoubleDom) -> yrwi_event_pull
//                                            (the doubleDomCache lives with the event)
//
// GpuReferenceOrder keeps SearchEvent.addRWIs in Java and only moves the ranking to
// the GPU; with this class the whole per-posting loop leaves the CPU: a container
// goes to the GPU as its RowSet bytes, and no per-posting Java work is left: a
// pulled entry becomes the WordReferenceVars Fulltext.getMetadata(element) reads
// (Fulltext.java:339-346) from the row the event's doublecheck set names for it
// (yrwi_event_source) -- for the pulled entries only.
//
// Wiring (INTEGRATION.md): SearchEvent.<init> opens one per event when a GpuRWI is
// configured; addRWIs and pullOneRWI delegate to it; cleanup() closes it (a dropped
// event returns its device memory through GpuRWI's reaper, GpuRWI.EventHandle: a
// phantom reference, Java 8 like YaCy's build).
package net.yacy.search.query;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.List;

import net.yacy.cora.document.encoding.ASCII;
import net.yacy.cora.document.id.DigestURL;
import net.yacy.cora.sorting.WeakPriorityBlockingQueue;
import net.yacy.kelondro.data.word.WordReference;
import net.yacy.kelondro.data.word.WordReferenceRow;
import net.yacy.kelondro.data.word.WordReferenceVars;
import net.yacy.kelondro.index.GpuRows;
import net.yacy.kelondro.rwi.GpuRWI;
import net.yacy.kelondro.rwi.ReferenceContainer;
import net.yacy.search.index.Segment;
import net.yacy.search.ranking.RankingProfile;

public final class GpuRWIStack implements AutoCloseable {

    private static final int ROW = 40;  // WordReferenceRow.urlEntryRow.objectsize

    private final GpuRWI gpu;
    private final long event;
    private final GpuRWI.EventHandle release;
    // every arrival's rows (the bytes given to the GPU, in arrival order) and whether it was local
    private final ArrayList<byte[]> rows = new ArrayList<byte[]>();
    private final ArrayList<Boolean> local = new ArrayList<Boolean>();
    private boolean closed = false;

    /**
     * @param k         rwiStack bound (max_results_rwi, SearchEvent.java:118)
     * @param maxPostings the most postings all arrivals together will bring (sizes the url set)
     * @param filter    the addRWIs constraints as GpuRWI.eventOpenFiltered takes them (QueryParams:
     *                  constraint, allofconstraint, contentdom, strict, modifier language, sitehash,
     *                  alternative sitehash, siteexcludes, the urlhashes already seen)
     */
    public GpuRWIStack(final GpuRWI gpu, final RankingProfile profile, final String targetLanguage, final int k,
                       final long maxPostings, final GpuRWI.EventFilter filter) {
        this.gpu = gpu;
        this.event = gpu.eventOpenFiltered(GpuRWI.profile32(profile), targetLanguage, System.currentTimeMillis(), k,
                                           maxPostings, filter);
        if (this.event == 0) throw new IllegalStateException("yrwi_event_open failed");
        this.release = gpu.track(this, this.event);
    }

    /** The addRWIs constraints of a query (SearchEvent.java:736-806) as the event takes
     *  them; the alternative site hash is SearchEvent's acceptableAlternativeSitehash
     *  (:716-718).  Urls SearchEvent already holds go in via filter.urlhashes. */
    public static GpuRWI.EventFilter filterOf(final QueryParams q) {
        final GpuRWI.EventFilter f = new GpuRWI.EventFilter();
        if (q.constraint != null) f.constraint = q.constraint.bytes();
        f.allOfConstraint = q.allofconstraint;
        f.contentdom = q.contentdom.getCode();
        f.strictContentDom = q.isStrictContentDom();
        f.modifierLanguage = q.modifier.language;
        if (q.modifier.sitehash != null) {
            f.sitehash = ASCII.getBytes(q.modifier.sitehash);
            if (q.modifier.sitehost != null && q.modifier.sitehost.length() > 0) {
                try {
                    f.altSitehash = ASCII.getBytes(DigestURL.hosthash(q.modifier.sitehost.startsWith("www.")
                        ? q.modifier.sitehost.substring(4) : "www." + q.modifier.sitehost, 80));
                } catch (final java.net.MalformedURLException e) {
                    f.altSitehash = null;  // as SearchEvent: no alternative then
                }
            }
        } else if (q.siteexcludes != null) {
            f.siteexcludes = new byte[q.siteexcludes.size()][];
            int i = 0;
            for (final String h : q.siteexcludes) f.siteexcludes[i++] = ASCII.getBytes(h);
        }
        return f;
    }

    /** SearchEvent.addRWIs(index, local, ...) for the posting loop (:673-836); the
     *  caller keeps the statistics it logs (local_rwi_stored / remote counters). */
    public synchronized int add(final ReferenceContainer<WordReference> container, final boolean isLocal) {
        final int n = container.size();
        if (n == 0 || this.closed) return 0;
        final byte[] r = GpuRows.sortedRows(container);  // the container's RowSet bytes, its order
        this.gpu.addRWIs(this.event, r, n, isLocal);
        this.rows.add(r);
        this.local.add(isLocal);
        return n;
    }

    /** SearchEvent.pullOneRWI(skipDoubleDom) up to maxn times: the entries in pull order,
     *  each the posting the doublecheck admitted for its url (yrwi_event_source: the
     *  url's first posting that passed the constraints, in whichever arrival) with its
     *  cardinal as weight. */
    public synchronized List<WeakPriorityBlockingQueue.Element<WordReferenceVars>> pull(final boolean skipDoubleDom,
                                                                                       final int maxn) {
        final ArrayList<WeakPriorityBlockingQueue.Element<WordReferenceVars>> out =
            new ArrayList<WeakPriorityBlockingQueue.Element<WordReferenceVars>>();
        if (this.closed || maxn <= 0) return out;
        final byte[] hits = this.gpu.pullRWI(this.event, skipDoubleDom, maxn);  // 24-byte yrwi_hit records
        if (hits == null || hits.length == 0) return out;
        final int n = hits.length / 24;
        final byte[] urls = new byte[12 * n];
        for (int h = 0; h < n; h++) System.arraycopy(hits, 24 * h, urls, 12 * h, 12);
        final int[] src = this.gpu.eventSource(this.event, urls, n);  // arrival (1-based), row per hit
        final ByteBuffer b = ByteBuffer.wrap(hits).order(ByteOrder.LITTLE_ENDIAN);
        for (int h = 0; h < n; h++) {
            final int a = src[2 * h] - 1, row = src[2 * h + 1];
            if (a < 0 || a >= this.rows.size()) continue;  // (cannot happen: every stack entry came from an arrival)
            final byte[] rb = new byte[ROW];
            System.arraycopy(this.rows.get(a), row * ROW, rb, 0, ROW);
            // (WordReferenceRow's Row.Entry constructor is protected: the factory's produceSlow)
            final WordReference wr = Segment.wordReferenceFactory.produceSlow(WordReferenceRow.urlEntryRow.newEntry(rb));
            out.add(new WeakPriorityBlockingQueue.ReverseElement<WordReferenceVars>(
                new WordReferenceVars(wr, this.local.get(a)), b.getLong(24 * h + 16)));
        }
        return out;
    }

    /** SearchEvent.flagcount and the admitted counts (yrwi_event_result's info). */
    public synchronized int[] flagCount() {
        return this.closed ? new int[32] : this.gpu.eventFlagCount(this.event);
    }

    @Override
    public synchronized void close() {
        if (!this.closed) {
            this.closed = true;
            this.release.release();
        }
    }
}
