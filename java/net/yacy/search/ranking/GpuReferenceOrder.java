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
// the racy reference), then each posting's cardinal is looked up.  The queue is
// returned complete and ends with WordReferenceVars.poison, as addRWIs expects.
package net.yacy.search.ranking;

import java.util.Arrays;
import java.util.HashMap;
import java.util.Iterator;
import java.util.Map;
import java.util.concurrent.BlockingQueue;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.LinkedBlockingQueue;

import net.yacy.cora.document.encoding.ASCII;
import net.yacy.kelondro.data.word.WordReference;
import net.yacy.kelondro.data.word.WordReferenceVars;
import net.yacy.kelondro.rwi.GpuRWI;
import net.yacy.kelondro.rwi.ReferenceContainer;

public class GpuReferenceOrder extends ReferenceOrder {

    private static final int EXPORT_HEADER = 14;  // RowCollection.exportOverheadSize (RowCollection.java:175)

    private final GpuRWI gpu;
    private final int[] profile32;
    private final String language;
    private final int coeffAuthority;
    // settled cardinal of every posting of the containers normalised so far, by url hash
    private final Map<String, Long> scores = new ConcurrentHashMap<String, Long>();
    // ReferenceOrder.doms / maxdomcount of the last container (authority, :176-216)
    private volatile Map<String, Integer> doms = new HashMap<String, Integer>();
    private volatile int maxdomcount = 0;

    public GpuReferenceOrder(final RankingProfile profile, final String language, final GpuRWI gpu) {
        super(profile, language);
        this.gpu = gpu;
        this.profile32 = GpuRWI.profile32(profile);
        this.language = language;
        this.coeffAuthority = profile.coeff_authority;
    }

    @Override
    public BlockingQueue<WordReferenceVars> normalizeWith(final ReferenceContainer<WordReference> container,
                                                          final long maxtime, final boolean local) {
        final LinkedBlockingQueue<WordReferenceVars> out = new LinkedBlockingQueue<WordReferenceVars>();
        final int m = container.size();
        if (m > 0) {
            // the RowSet chunkcache: sorted 40-byte WordReferenceRow rows after the export header
            final byte[] exported = container.exportCollection();
            final byte[] rows = Arrays.copyOfRange(exported, EXPORT_HEADER, EXPORT_HEADER + m * 40);
            final long[] sc = this.gpu.normalizeScore(rows, m, this.profile32, this.language, System.currentTimeMillis());
            final Map<String, Integer> d = new HashMap<String, Integer>();
            int maxd = 0;
            final Iterator<WordReference> i = container.entries();
            int p = 0;
            while (i.hasNext()) {
                final WordReferenceVars v = new WordReferenceVars(i.next(), local);
                this.scores.put(ASCII.String(v.urlhash()), sc[p++]);
                if (this.coeffAuthority > 12) {
                    final String h = v.hosthash();
                    final int c = d.containsKey(h) ? d.get(h) + 1 : 1;
                    d.put(h, c);
                    if (c > maxd) maxd = c;
                }
                out.add(v);
            }
            this.doms = d;
            this.maxdomcount = maxd;
        }
        out.add(WordReferenceVars.poison);
        return out;
    }

    @Override
    public int authority(final String hostHash) {
        final Integer c = this.doms.get(hostHash);
        return ((c == null ? 0 : c) << 8) / (1 + this.maxdomcount);
    }

    @Override
    public long cardinal(final WordReference t) {
        final Long s = this.scores.get(ASCII.String(t.urlhash()));
        if (s == null) throw new IllegalStateException("cardinal of a posting that was not normalised");
        return s;
    }
}
