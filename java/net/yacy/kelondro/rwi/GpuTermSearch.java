// GpuTermSearch.java -- TermSearch / joinExcludeContainers on the GPU-resident
// index of libyrwi (SURVEY.md §8b drop-in; UNVERIFIED: no JDK in this image).
//
// Replaces (paths relative to source/net/yacy):
//   kelondro/rwi/TermSearch.java:42-70              -> GpuTermSearch(...) / joined()
//   kelondro/rwi/ReferenceContainer.java:310-326    -> joinExcludeContainers(...)
// Wiring: AbstractIndex.query (AbstractIndex.java:130-137) returns
//   new TermSearch<R>(...)
// today; with a GPU index the TermSearch constructor's join (TermSearch.java:65-69)
// becomes GpuTermSearch.joinExclude(gpu, factory, queryHashes, excludeHashes,
// maxDistance) -- INTEGRATION.md shows the six-line patch.  The include/exclude
// lists are the GPU index's own (put there by IndexCell.add / loadHeaps), so no
// container crosses PCIe on the query path; only the joined rows come back.
package net.yacy.kelondro.rwi;

import java.util.Collection;
import java.util.Iterator;

import net.yacy.cora.storage.HandleSet;
import net.yacy.kelondro.data.word.WordReferenceRow;
import net.yacy.kelondro.index.RowSet;

public final class GpuTermSearch {

    private GpuTermSearch() {}

    /** TermSearch's joined container for the query's include / exclude word hashes
     *  (HandleSets: sorted sets of 12-byte hashes), joined on the GPU index.  An empty
     *  container when any include word is unknown (AbstractIndex.java:108-127). */
    public static <R extends Reference> ReferenceContainer<R> joinExclude(
            final GpuRWI gpu, final ReferenceFactory<R> factory, final HandleSet queryHashes,
            final HandleSet excludeHashes, final int maxDistance) {
        final byte[] rows = gpu.joinExclude(toArray(queryHashes), toArray(excludeHashes), maxDistance,
                                            System.currentTimeMillis());
        return wrap(factory, rows);
    }

    /** ReferenceContainer.joinExcludeContainers for containers that live on the CPU
     *  (e.g. a remote peer's): they are put into `scratch` (a GpuRWI context used only
     *  for this) under their term hashes, joined there and removed again. */
    public static <R extends Reference> ReferenceContainer<R> joinExcludeContainers(
            final GpuRWI scratch, final ReferenceFactory<R> factory,
            final Collection<ReferenceContainer<R>> includeContainers,
            final Collection<ReferenceContainer<R>> excludeContainers, final int maxDistance) {
        if (includeContainers == null) return ReferenceContainer.emptyContainer(factory, null);
        final byte[][] inc = put(scratch, includeContainers);
        final byte[][] exc = put(scratch, excludeContainers);
        try {
            return wrap(factory, scratch.joinExclude(inc, exc, maxDistance, System.currentTimeMillis()));
        } finally {
            for (final byte[] t : inc) scratch.putList(t, new byte[0], 0);
            for (final byte[] t : exc) scratch.putList(t, new byte[0], 0);
        }
    }

    private static <R extends Reference> byte[][] put(final GpuRWI scratch,
                                                     final Collection<ReferenceContainer<R>> cs) {
        if (cs == null) return new byte[0][];
        final byte[][] terms = new byte[cs.size()][];
        int i = 0;
        for (final ReferenceContainer<R> c : cs) {
            final byte[] exported = c.exportCollection();
            final int n = c.size();
            final byte[] rows = new byte[n * 40];
            if (n > 0) System.arraycopy(exported, 14, rows, 0, n * 40);  // RowCollection.exportOverheadSize
            scratch.putList(c.getTermHash(), rows, n);
            terms[i++] = c.getTermHash();
        }
        return terms;
    }

    private static <R extends Reference> ReferenceContainer<R> wrap(final ReferenceFactory<R> factory,
                                                                   final byte[] rows) {
        final int m = rows == null ? 0 : rows.length / 40;
        if (m == 0) return ReferenceContainer.emptyContainer(factory, null);
        // the rows are sorted by url hash: sortBound = m
        return new ReferenceContainer<R>(factory, null, new RowSet(WordReferenceRow.urlEntryRow, m, rows, m));
    }

    private static byte[][] toArray(final HandleSet hs) {
        if (hs == null) return new byte[0][];
        final byte[][] a = new byte[hs.size()][];
        final Iterator<byte[]> i = hs.iterator();
        int k = 0;
        while (i.hasNext()) a[k++] = i.next();
        return a;
    }
}
