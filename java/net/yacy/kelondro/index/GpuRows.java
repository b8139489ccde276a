// GpuRows.java -- a RowCollection's own row bytes for libyrwi, without a Java-side copy
// (SURVEY.md §8b drop-in; UNVERIFIED: no JDK in this image).
//
// RowCollection keeps its rows in one byte[] (`chunkcache`, protected,
// kelondro/index/RowCollection.java:68-70): `size()` rows of
// `rowdef.objectsize` bytes, the first `sortBound` of them sorted.  This class
// lives in the same package, so the GPU drop-ins can hand that array to JNI
// itself instead of exportCollection() (a full copy with a 14-byte header,
// RowCollection.java:175-231) plus Arrays.copyOfRange (a second copy).  The JNI
// side then copies the first n * 40 bytes once into native memory
// (GetByteArrayRegion in yrwi_jni.c copy_in: no critical region is held across
// library calls that wait for the GPU, so the collector is never blocked).
package net.yacy.kelondro.index;

public final class GpuRows {

    private GpuRows() {}

    /** The collection's backing rows, sorted first (RowCollection.sort, :684 -- a
     *  no-op when sortBound == size, as for the GPU join's output and the index's
     *  own containers).  The first c.size() * c.row().objectsize bytes are the
     *  rows in url-hash order; the array is the collection's own: read only. */
    public static byte[] sortedRows(final RowCollection c) {
        c.sort();
        return c.chunkcache;
    }
}
