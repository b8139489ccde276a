// GpuReferenceOrder.java -- ReferenceOrder whose normalisation and scoring run in
// libyrwi on the GPU (SURVEY.md §8b drop-in; UNVERIFIED: no JDK in this image).
//
// Replaces (paths relative to source/net/yacy):
//   search/ranking/ReferenceOrder.java:70-79   normalizeWith -> one yrwi_normalize_score call
//   search/ranking/ReferenceOrder.java:213-216 authority     -> host counts of the last container
//   search/ranking/ReferenceOrder.java:223-265 cardinal      -> the settled score of that posting
// Wiring: SearchEvent.<init> (SearchEvent.java:436) constructs
//   new GpuReferenceOrder(query.ranking, query.targetlang, gpu)
// instead of new ReferenceOrder(...); SearchEvent.addRWIs is unchanged.
//
// Semantics: every container handed to normalizeWith is normalised over itself
// with settled min/max (DESIGN.md §2: the canonical, deterministic reading of
// the racy reference), then each posting's cardinal is read back.  The queue is
// returned complete and ends with WordReferenceVars.poison, as addRWIs expects.
//
// Per container this class makes no copy of the rows (the RowSet's own byte[]
// goes to JNI, GpuRows), keeps the scores in one long[] in container order, and
// each queued entry carries its position in it (Entry), so cardinal(e) is an
// array read: no per-posting key String and no map.  The host counts behind
// authority() are built only if something asks for them (the inherited
// cardinal(URIMetadataNode)); the GPU scores already include authority.
package net.yacy.search.ranking;

import java.util.HashMap;
import java.util.Iterator;
import java.util.Map;
import java.util.concurrent.BlockingQueue;
import java.util.concurrent.LinkedBlockingQueue;

import net.yacy.cora.document.encoding.ASCII;
import net.yacy.kelondro.data.word.WordReference;
import net.yacy.kelondro.data.word.WordReferenceVars;
import net.yacy.kelondro.index.GpuRows;
import net.yacy.kelondro.rwi.GpuRWI;
import net.yacy.kelondro.rwi.ReferenceContainer;

public class GpuReferenceOrder extends ReferenceOrder {

    private static final int ROW = 40;  // WordReferenceRow.urlEntryRow.objectsize

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
    private final int[] profile32;
    private final String language;
    // the last normalised container's rows (authority() counts its hosts on demand)
    private volatile byte[] lastRows = null;
    private volatile int lastCount = 0;
    private Map<String, Integer> doms = null;
    private int maxdomcount = 0;

    public GpuReferenceOrder(final RankingProfile profile, final String language, final GpuRWI gpu) {
        super(profile, language);
        this.gpu = gpu;
        this.profile32 = GpuRWI.profile32(profile);
        this.language = language;
    }

    @Override
    public BlockingQueue<WordReferenceVars> normalizeWith(final ReferenceContainer<WordReference> container,
                                                          final long maxtime, final boolean local) {
        final LinkedBlockingQueue<WordReferenceVars> out = new LinkedBlockingQueue<WordReferenceVars>();
        final int m = container.size();
        if (m > 0) {
            // RowSet.chunkcache: the sorted 40-byte WordReferenceRow rows, handed over as they are
            final byte[] rows = GpuRows.sortedRows(container);
            final long[] sc = this.gpu.normalizeScore(rows, m, this.profile32, this.language, System.currentTimeMillis());
            final Iterator<WordReference> i = container.entries();  // the same (sorted) row order
            int p = 0;
            while (i.hasNext()) out.add(new Entry(i.next(), local, sc, p++));
            synchronized (this) {
                this.lastRows = rows;
                this.lastCount = m;
                this.doms = null;
            }
        }
        out.add(WordReferenceVars.poison);
        return out;
    }

    @Override
    public synchronized int authority(final String hostHash) {
        if (this.doms == null) {  // host counts of the last container (ReferenceOrder.java:176-182)
            final Map<String, Integer> d = new HashMap<String, Integer>();
            int maxd = 0;
            final byte[] rows = this.lastRows;
            for (int r = 0; rows != null && r < this.lastCount; r++) {
                final String h = ASCII.String(rows, r * ROW + 6, 6);  // url-hash chars 6..11
                final Integer c0 = d.get(h);
                final int c = c0 == null ? 1 : c0 + 1;
                d.put(h, c);
                if (c > maxd) maxd = c;
            }
            this.doms = d;
            this.maxdomcount = maxd;
        }
        final Integer c = this.doms.get(hostHash);
        return ((c == null ? 0 : c) << 8) / (1 + this.maxdomcount);
    }

    @Override
    public long cardinal(final WordReference t) {
        if (t instanceof Entry) return ((Entry) t).score();
        throw new IllegalStateException("cardinal of a posting that was not normalised by this order");
    }
}
