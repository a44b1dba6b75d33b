package dev.zarr.zarrjava.hip;

/**
 * JNI entry points of libzarrhip_jni.so (zarr-java_amd/java/jni/zarrhip_jni.c), which
 * forwards to the zarrhip C-ABI (include/zarrhip.h).  A status of 3 (ZH_EUNSUPPORTED)
 * means "codec chain not device-supported": callers fall back to the reference codec.
 * Data errors surface as dev.zarr.zarrjava.ZarrException with the reference's messages.
 *
 * Devices: ZH_DEVICES="0,1,...,7" spreads every region read over those GPUs
 * (zh_array_read_multi: one slab per device, each copied straight into its slice of the
 * result); otherwise ZH_DEVICE (default 0) is the one device.
 *
 * The codec path (HipShardingIndexedCodec, one shard per call) is called concurrently by
 * core.Array.read's ForkJoin threads (M/core/Array.java:403-407).  A zh_ctx serialises its
 * calls on its own stream, so those threads draw from a pool of ZH_CODEC_CONTEXTS contexts on
 * the first device (default 4): each ForkJoin thread keeps one, and the shards' H2D, decode
 * and D2H overlap across contexts instead of queueing on one.
 */
public final class ZarrHip {
    public static final int UNSUPPORTED = 3;

    private static final boolean AVAILABLE;
    private static final long[] CTXS;
    private static final long[] CODEC_POOL;
    private static final java.util.concurrent.atomic.AtomicInteger NEXT =
            new java.util.concurrent.atomic.AtomicInteger();
    private static final ThreadLocal<Long> CODEC_CTX = ThreadLocal.withInitial(
            () -> CODEC_POOL[Math.floorMod(NEXT.getAndIncrement(), CODEC_POOL.length)]);

    static {
        long[] ctxs = new long[0];
        if (!"1".equals(System.getenv("ZH_DISABLE"))) {
            try {
                System.loadLibrary("zarrhip_jni");
                String list = System.getenv("ZH_DEVICES");
                if (list == null) {
                    String dev = System.getenv("ZH_DEVICE");
                    list = dev == null ? "0" : dev;
                }
                String[] ids = list.split(",");
                ctxs = new long[ids.length];
                for (int i = 0; i < ids.length; i++) {
                    ctxs[i] = ctxCreate(Integer.parseInt(ids[i].trim()));
                    if (ctxs[i] == 0) {
                        ctxs = new long[0];
                        break;
                    }
                }
            } catch (Throwable t) {
                ctxs = new long[0];
            }
        }
        AVAILABLE = ctxs.length > 0;
        CTXS = ctxs;
        long[] pool = ctxs.length > 0 ? new long[]{ctxs[0]} : new long[0];
        if (ctxs.length > 0) {
            String n = System.getenv("ZH_CODEC_CONTEXTS");
            int want = 4;
            try {
                if (n != null) want = Math.max(1, Integer.parseInt(n.trim()));
            } catch (NumberFormatException e) {
                want = 4;
            }
            String list = System.getenv("ZH_DEVICES");
            if (list == null) list = System.getenv("ZH_DEVICE") == null ? "0" : System.getenv("ZH_DEVICE");
            int dev0 = Integer.parseInt(list.split(",")[0].trim());
            java.util.List<Long> extra = new java.util.ArrayList<>();
            extra.add(ctxs[0]);
            for (int i = 1; i < want; i++) {
                long c = ctxCreate(dev0);
                if (c == 0) break;
                extra.add(c);
            }
            pool = new long[extra.size()];
            for (int i = 0; i < pool.length; i++) pool[i] = extra.get(i);
        }
        CODEC_POOL = pool;
    }

    private ZarrHip() {
    }

    public static boolean available() {
        return AVAILABLE;
    }

    static long ctx() {
        return CTXS[0];
    }

    static long[] ctxs() {
        return CTXS;
    }

    /** The calling thread's context of the codec pool (see the class comment). */
    static long codecCtx() {
        return CODEC_CTX.get();
    }

    static native long ctxCreate(int device);

    static native void ctxDestroy(long ctx);

    /** core.Array.read(offset, shape) for all chunks of the region in one device call. */
    static native int arrayRead(long ctx, int[] meta, long[] shape, int[] chunkShape,
                                int[] innerShape, int[] order, byte[] fill, byte[][] chunks,
                                long[] offset, long[] regionShape, Object out);

    /** The same read split into one slab per device context (zh_array_read_multi). */
    static native int arrayReadMulti(long[] ctxs, int[] meta, long[] shape, int[] chunkShape,
                                     int[] innerShape, int[] order, byte[] fill, byte[][] chunks,
                                     long[] offset, long[] regionShape, Object out);

    /**
     * core.Array.write of a region of whole chunks (clipped only by the array boundary):
     * the encoded chunk objects in computeChunkCoords order, null entries for chunks that are
     * all fill_value (delete the key); null when the chain or region is not device-supported.
     */
    static native byte[][] arrayWrite(long ctx, int[] meta, long[] shape, int[] chunkShape,
                                      int[] innerShape, int[] order, byte[] fill, long[] offset,
                                      long[] regionShape, Object data);

    /**
     * core.Array.write of a region of whole chunks into a FilesystemStore
     * (zh_array_write_files): paths[i] is StoreHandle.toPath() of the i-th chunk of
     * computeChunkCoords, storeRoot / storeName the store's directory and toString() (the
     * StoreException text names them); the library encodes on the device and writes (all
     * fill_value: deletes) the chunk files.  Returns 0, or UNSUPPORTED when the caller must
     * write itself.
     */
    static native int arrayWriteFiles(long ctx, int[] meta, long[] shape, int[] chunkShape,
                                      int[] innerShape, int[] order, byte[] fill, long[] offset,
                                      long[] regionShape, Object data, String storeRoot,
                                      String storeName, String[] paths);

    /** ShardingIndexedCodec.decodePartial over one shard's bytes. */
    static native int shardDecodePartial(long ctx, int[] meta, long[] shape, int[] chunkShape,
                                         int[] innerShape, int[] order, byte[] fill, byte[] shard,
                                         long[] offset, int[] partShape, Object out);

    /**
     * zh_shard_ranges: the (offset, nbytes) pairs of the stored shard a part references, read
     * from its stored index, adjacent ranges merged up to maxRun bytes (0: one per inner
     * chunk).  checkIndex: first zh_shard_index_check (the index crc32c on the host; a mismatch
     * throws the reference's ZarrException); otherwise the device checks it.
     */
    static native long[] shardRanges(int[] meta, long[] shape, int[] chunkShape,
                                     int[] innerShape, int[] order, byte[] fill, byte[] index,
                                     long shardSize, long[] partLo, long[] partHi, long maxRun,
                                     boolean checkIndex) throws dev.zarr.zarrjava.ZarrException;

    /**
     * core.Array.read over shards given as stored index + pieces (zh_array_read_pieces; with
     * several contexts zh_array_read_pieces_multi).  Per shard i: indexes[i] (null: whole in
     * piece 0, or missing when it has no pieces), sizes[i] (-1 unknown), and its pieces.
     */
    static native int arrayReadPieces(long[] ctxs, int[] meta, long[] shape, int[] chunkShape,
                                      int[] innerShape, int[] order, byte[] fill,
                                      byte[][] indexes, long[] sizes, long[][] pieceOffsets,
                                      long[][] pieceLens, byte[][][] pieceData, long[] offset,
                                      long[] regionShape, Object out);

    /**
     * core.Array.read over a FilesystemStore (zh_array_read_files; with several contexts
     * zh_array_read_files_multi, one slab per device): paths[i] is
     * StoreHandle.toPath() of the i-th chunk of computeChunkCoords (null: no key); the library
     * reads the files (exists, the index and the referenced ranges, or whole chunks) with the
     * pipelined read, so no chunk bytes cross into the Java heap.  An unreadable file throws
     * dev.zarr.zarrjava.store.StoreException naming storeName (FilesystemStore.toString())
     * and the key below storeRoot (the store's directory).
     */
    static native int arrayReadFiles(long[] ctxs, int[] meta, long[] shape, int[] chunkShape,
                                     int[] innerShape, int[] order, byte[] fill,
                                     String storeRoot, String storeName, String[] paths,
                                     long[] offset, long[] regionShape, Object out);

    /** The directory of a FilesystemStore (its keys resolve below it). */
    static String storeRoot(dev.zarr.zarrjava.store.Store store) {
        return new dev.zarr.zarrjava.store.StoreHandle(store).toPath().toString();
    }

    /** ShardingIndexedCodec.decodePartial over one shard as index + pieces. */
    static native int shardDecodePieces(long ctx, int[] meta, long[] shape, int[] chunkShape,
                                        int[] innerShape, int[] order, byte[] fill, byte[] index,
                                        long size, long[] pieceOffsets, long[] pieceLens,
                                        byte[][] pieceData, long[] offset, int[] partShape,
                                        Object out);

    // ---- flattening of ShardPieces[] into the JNI's arrays (null entries: missing shards)
    static byte[][] indexes(ShardPieces[] s) {
        byte[][] r = new byte[s.length][];
        for (int i = 0; i < s.length; i++) r[i] = s[i] == null ? null : s[i].index;
        return r;
    }

    static long[] sizes(ShardPieces[] s) {
        long[] r = new long[s.length];
        for (int i = 0; i < s.length; i++) r[i] = s[i] == null ? -1 : s[i].shardSize;
        return r;
    }

    static long[][] pieceOffsets(ShardPieces[] s) {
        long[][] r = new long[s.length][];
        for (int i = 0; i < s.length; i++) r[i] = s[i] == null ? new long[0] : s[i].offsets;
        return r;
    }

    static long[][] pieceLens(ShardPieces[] s) {
        long[][] r = new long[s.length][];
        for (int i = 0; i < s.length; i++) r[i] = s[i] == null ? new long[0] : s[i].storedLens;
        return r;
    }

    static byte[][][] pieceData(ShardPieces[] s) {
        byte[][][] r = new byte[s.length][][];
        for (int i = 0; i < s.length; i++) r[i] = s[i] == null ? new byte[0][] : s[i].data;
        return r;
    }
}
