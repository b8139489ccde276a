// GpuTermSearch.java -- TermSearch over the GPU-resident index of libyrwi
// (SURVEY.md §8b drop-in; UNVERIFIED: no JDK in this image).
//
// Replaces (paths relative to source/net/yacy):
//   kelondro/rwi/TermSearch.java:42-70            -> GpuTermSearch(...): no CPU container is fetched
//   kelondro/rwi/AbstractIndex.java:96-128        -> J1 existence from the GPU index's list sizes
//   kelondro/rwi/ReferenceContainer.java:310-326  -> the join, one yrwi_join_exclude call
//   kelondro/rwi/TermSearch.java:76-78 inclusion() -> fetched from the GPU index only when asked
// Wiring: AbstractIndex.query (AbstractIndex.java:130-137) returns
//   gpu == null ? new TermSearch<R>(...) : new GpuTermSearch<R>(gpu, ...)
// and TermSearch gets a protected constructor for subclasses (INTEGRATION.md).
//
// The reference's TermSearch runs base.searchConjunction for every include and
// exclude word (TermSearch.java:50-62): IndexCell.get, i.e. RAM cache merged
// with the BLOB heaps and a clone per row, on every query -- then joins them.
// Here the lists are the GPU index's own (IndexCell.add / loadHeaps put them
// there): existence and sizes come from yrwi_list_size, the join runs on the
// device, and only the joined rows cross PCIe.  inclusion() -- which SearchEvent
// reads only to build index abstracts (SearchEvent.java:505-531, via
// searchContainerMap :2476) -- is materialised from the GPU lists on first use;
// abstracts()/inclusionSizes() serve that caller without any container at all.
package net.yacy.kelondro.rwi;

import java.util.Collection;
import java.util.Iterator;
import java.util.TreeMap;

import net.yacy.cora.order.Base64Order;
import net.yacy.cora.storage.HandleSet;
import net.yacy.kelondro.data.word.WordReferenceRow;
import net.yacy.kelondro.index.GpuRows;
import net.yacy.kelondro.index.RowSet;

public class GpuTermSearch<ReferenceType extends Reference> extends TermSearch<ReferenceType> {

    private final GpuRWI gpu;
    private final ReferenceFactory<ReferenceType> factory;
    private final byte[][] include;
    private final long[] sizes;      // GPU list size of every include word
    private final boolean complete;  // every include word has a non-empty list (J1)
    private TreeMap<byte[], ReferenceContainer<ReferenceType>> inclusionContainers = null;

    /** TermSearch(base, queryHashes, excludeHashes, urlselection, termFactory, maxDistance)
     *  on the GPU index.  A non-null urlselection restricts every include and exclude
     *  list to those urls before the conjunction, as ReferenceContainerCache.get(key,
     *  urlselection) does (the local search passes null, SearchEvent.java:619; IndexCell
     *  ignores the argument).  inclusion() / sizes stay the unrestricted lists'. */
    public GpuTermSearch(final GpuRWI gpu, final HandleSet queryHashes, final HandleSet excludeHashes,
                         final HandleSet urlselection, final ReferenceFactory<ReferenceType> termFactory,
                         final int maxDistance) {
        super(join(gpu, queryHashes, excludeHashes, urlselection, termFactory, maxDistance));
        this.gpu = gpu;
        this.factory = termFactory;
        this.include = toArray(queryHashes);
        this.sizes = gpu.listSizes(this.include);
        boolean all = this.include.length > 0;
        for (final long n : this.sizes) if (n == 0) all = false;
        this.complete = all;
    }

    // J1 (AbstractIndex.java:108-127, TermSearch.java:50-62: a missing include word
    // empties the result, exclude words count only when all include words exist)
    // and the join: both inside yrwi_join_exclude
    private static <R extends Reference> ReferenceContainer<R> join(
            final GpuRWI gpu, final HandleSet queryHashes, final HandleSet excludeHashes, final HandleSet urlselection,
            final ReferenceFactory<R> termFactory, final int maxDistance) {
        if (queryHashes == null || queryHashes.isEmpty()) return ReferenceContainer.emptyContainer(termFactory, null);
        if (urlselection != null)
            return wrap(termFactory, gpu.termSearch(toArray(queryHashes), toArray(excludeHashes), toArray(urlselection),
                                                    maxDistance, System.currentTimeMillis()));
        return wrap(termFactory, gpu.joinExclude(toArray(queryHashes), toArray(excludeHashes), maxDistance,
                                                 System.currentTimeMillis()));
    }

    /** The include words' containers (TermSearch.inclusion), read from the GPU index
     *  on the first call only; empty when an include word has no list. */
    @Override
    public synchronized TreeMap<byte[], ReferenceContainer<ReferenceType>> inclusion() {
        if (this.inclusionContainers == null) {
            final TreeMap<byte[], ReferenceContainer<ReferenceType>> m =
                    new TreeMap<byte[], ReferenceContainer<ReferenceType>>(Base64Order.enhancedCoder);
            if (this.complete) {
                for (final byte[] t : this.include) {
                    final byte[] rows = this.gpu.getList(t);
                    final int n = rows.length / 40;
                    m.put(t, new ReferenceContainer<ReferenceType>(this.factory, t,
                            new RowSet(WordReferenceRow.urlEntryRow, n, rows, n)));
                }
            }
            this.inclusionContainers = m;
        }
        return this.inclusionContainers;
    }

    /** container.size() of every inclusion() entry (SearchEvent.java:519-530 IACount), without the containers. */
    public TreeMap<byte[], Long> inclusionSizes() {
        final TreeMap<byte[], Long> m = new TreeMap<byte[], Long>(Base64Order.enhancedCoder);
        if (this.complete) for (int i = 0; i < this.include.length; i++) m.put(this.include[i], this.sizes[i]);
        return m;
    }

    /** WordReferenceFactory.compressIndex(container, null, 1000) of every inclusion()
     *  entry (SearchEvent.java:530 IAResults), computed on the device (yrwi_index_abstracts). */
    public TreeMap<byte[], String> abstracts(final long capacity) {
        final TreeMap<byte[], String> m = new TreeMap<byte[], String>(Base64Order.enhancedCoder);
        if (!this.complete) return m;
        final String[] a = this.gpu.indexAbstracts(this.include, capacity);
        for (int i = 0; i < a.length; i++) m.put(this.include[i], a[i]);
        return m;
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
            // the RowSet's own sorted rows (no exportCollection copy)
            scratch.putList(c.getTermHash(), GpuRows.sortedRows(c), c.size());
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
