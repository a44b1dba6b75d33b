package dev.zarr.zarrjava.hip;

/**
 * JNI entry points of libzarrhip_jni.so (zarr-java_amd/java/jni/zarrhip_jni.c), which
 * forwards to the zarrhip C-ABI (include/zarrhip.h).  A status of 3 (ZH_EUNSUPPORTED)
 * means "codec chain not device-supported": callers fall back to the reference codec.
 * Data errors surface as dev.zarr.zarrjava.ZarrException with the reference's messages.
 */
public final class ZarrHip {
    public static final int UNSUPPORTED = 3;

    private static final boolean AVAILABLE;
    private static final long CTX;

    static {
        boolean ok = false;
        long ctx = 0;
        if (!"1".equals(System.getenv("ZH_DISABLE"))) {
            try {
                System.loadLibrary("zarrhip_jni");
                String dev = System.getenv("ZH_DEVICE");
                ctx = ctxCreate(dev == null ? 0 : Integer.parseInt(dev));
                ok = ctx != 0;
            } catch (Throwable t) {
                ok = false;
            }
        }
        AVAILABLE = ok;
        CTX = ctx;
    }

    private ZarrHip() {
    }

    public static boolean available() {
        return AVAILABLE;
    }

    static long ctx() {
        return CTX;
    }

    static native long ctxCreate(int device);

    static native void ctxDestroy(long ctx);

    /** core.Array.read(offset, shape) for all chunks of the region in one device call. */
    static native int arrayRead(long ctx, int[] meta, long[] shape, int[] chunkShape,
                                int[] innerShape, int[] order, byte[] fill, byte[][] chunks,
                                long[] offset, long[] regionShape, Object out);

    /** ShardingIndexedCodec.decodePartial over one shard's bytes. */
    static native int shardDecodePartial(long ctx, int[] meta, long[] shape, int[] chunkShape,
                                         int[] innerShape, int[] order, byte[] fill, byte[] shard,
                                         long[] offset, int[] partShape, Object out);
}
