// GpuReferenceOrder.java -- ReferenceOrder whose normalisation and scoring run in
// libyrwi on the GPU (SURVEY.md §8b drop-in; UNVERIFIED: no JDK in this image).
//
// Replaces (paths relative to source/net/yacy):
//   search/ranking/ReferenceOrder.java:70-79,163-210  normalizeWith -> yrwi_event_order on the order's event
//   search/ranking/ReferenceOrder.java:213-216        authority     -> yrwi_event_authority (accumulated doms)
//   search/ranking/ReferenceOrder.java:223-265        cardinal      -> the posting's score from that call
// Wiring: SearchEvent.<init> (SearchEvent.java:436) constructs
//   new GpuReferenceOrder(query.ranking, query.targetlang, gpu)
// instead of new ReferenceOrder(...), and SearchEvent.cleanup() closes it;
// SearchEvent.addRWIs is unchanged.
//
// Semantics: YaCy keeps ONE ReferenceOrder per SearchEvent, and every container
// handed to normalizeWith continues it: min/max are cloned from the first posting
// ever seen and only folded afterwards (ReferenceOrder.java:173-174), the host
// counts accumulate in doms / maxdomcount (:196-198).  The local container
// (SearchEvent.java:631), a sitehost retry (:651), every remote peer's container
// (Protocol.java:802) and heuristic injections (Segment.java:758) are all scored
// against that accumulated state.  This class holds one libyrwi search event for
// the order's lifetime and hands it each container (yrwi_event_order): the same
// accumulation on the GPU, each posting scored under the state after its own
// container has been folded in (the settled reading of DESIGN.md §2; the
// reference races the workers' min/max updates against cardinal()).  The queue is
// returned complete and ends with WordReferenceVars.poison, as addRWIs expects.
//
// Per container this class hands the RowSet's own byte[] to JNI (GpuRows: no
// exportCollection copy on the Java side; the JNI copies it once into native
// memory, yrwi_jni.c copy_in), keeps the scores in one long[] in container order, and
// each queued entry carries its position in it (Entry), so cardinal(e) is an
// array read: no per-posting key String and no map.  authority() asks the GPU's
// accumulated host counts (they exist when coeff_authority > 12, the only case in
// which cardinal uses them); its answers are cached until the next container
// changes the counts, so the result workers' per-node calls (cardinal(
// URIMetadataNode)) reach the GPU once per distinct host.
//
// Resources: the event is order-only (yrwi_event_open_order: the state and a host
// table sized by expected hosts, no url set or stack), its device block reused
// from closed orders (no device-wide allocation per SearchEvent).  close() returns
// it; a SearchEvent that is dropped without cleanup() still returns it through
// GpuRWI's reaper (a phantom reference, GpuRWI.EventHandle: Java 8, YaCy's level).
// Every native call goes through GpuRWI, which serialises them on the shared
// context (a context is not thread-safe).
package net.yacy.search.ranking;

import java.util.HashMap;
import java.util.Iterator;
import java.util.concurrent.BlockingQueue;
import java.util.concurrent.LinkedBlockingQueue;

import net.yacy.cora.document.encoding.ASCII;
import net.yacy.kelondro.data.word.WordReference;
import net.yacy.kelondro.data.word.WordReferenceVars;
import net.yacy.kelondro.index.GpuRows;
import net.yacy.kelondro.rwi.GpuRWI;
import net.yacy.kelondro.rwi.ReferenceContainer;

public class GpuReferenceOrder extends ReferenceOrder implements AutoCloseable {

    /** Distinct hosts one SearchEvent's order is expected to see (the event's first
     *  host table, 12 B per slot, two slots per host: 3 MB); more hosts grow the
     *  table (yrwi_event_order), as ReferenceOrder.doms is unbounded. */
    public static final long DEFAULT_MAX_HOSTS = 1L << 17;

    /** A queued posting with its position in the container's score array. */
    public static final class Entry extends WordReferenceVars {
        private final long[] scores;
        private final int pos;

        Entry(final WordReference e, final boolean local, final long[] scores, final int pos) {
            super(e, local);
            this.scores = scores;
            this.pos = pos;
        }

        public long score() {
            return this.scores[this.pos];
        }
    }

    private final GpuRWI gpu;
    private long event;  // yrwi_event*: this order's ReferenceOrder state on the GPU
    private final GpuRWI.EventHandle release;  // returns the event, also if the order is dropped unclosed
    private final boolean authorityProfile;
    private final HashMap<String, Integer> authorityCache = new HashMap<String, Integer>();

    public GpuReferenceOrder(final RankingProfile profile, final String language, final GpuRWI gpu) {
        this(profile, language, gpu, DEFAULT_MAX_HOSTS);
    }

    public GpuReferenceOrder(final RankingProfile profile, final String language, final GpuRWI gpu,
                             final long maxHosts) {
        super(profile, language);
        this.gpu = gpu;
        this.authorityProfile = profile.coeff_authority > 12;
        // "now" is fixed for the event's lifetime (the clone's virtualAge clamp, J6)
        this.event = gpu.eventOpenOrder(GpuRWI.profile32(profile), language, System.currentTimeMillis(), maxHosts);
        if (this.event == 0) throw new IllegalStateException("yrwi_event_open_order failed");
        this.release = gpu.track(this, this.event);
    }

    @Override
    public BlockingQueue<WordReferenceVars> normalizeWith(final ReferenceContainer<WordReference> container,
                                                          final long maxtime, final boolean local) {
        final LinkedBlockingQueue<WordReferenceVars> out = new LinkedBlockingQueue<WordReferenceVars>();
        final int m = container.size();
        if (m > 0) {
            // RowSet.chunkcache: the container's 40-byte WordReferenceRow rows in its order
            final byte[] rows = GpuRows.sortedRows(container);
            final long[] sc;
            synchronized (this) {  // containers fold into the order one after another
                sc = this.gpu.eventOrder(this.event, rows, m, local);
                this.authorityCache.clear();  // the host counts changed
            }
            final Iterator<WordReference> i = container.entries();  // the same row order
            int p = 0;
            while (i.hasNext()) out.add(new Entry(i.next(), local, sc, p++));
        }
        out.add(WordReferenceVars.poison);
        return out;
    }

    @Override
    public synchronized int authority(final String hostHash) {
        if (!this.authorityProfile) return 0;  // no host counts: ReferenceOrder's doms stay empty
        final Integer a = this.authorityCache.get(hostHash);
        if (a != null) return a.intValue();
        final int v = this.gpu.eventAuthority(this.event, ASCII.getBytes(hostHash));
        this.authorityCache.put(hostHash, v);
        return v;
    }

    @Override
    public long cardinal(final WordReference t) {
        if (t instanceof Entry) return ((Entry) t).score();
        throw new IllegalStateException("cardinal of a posting that was not normalised by this order");
    }

    @Override
    public synchronized void close() {
        if (this.event != 0) {
            this.event = 0;
            this.release.release();  // once: the event back to the context
        }
    }
}
