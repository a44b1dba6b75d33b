package dev.zarr.zarrjava.hip;

import dev.zarr.zarrjava.ZarrException;
import dev.zarr.zarrjava.core.ArrayMetadata.CoreArrayMetadata;
import dev.zarr.zarrjava.core.codec.BytesBytesCodec;
import dev.zarr.zarrjava.v3.codec.Codec;
import dev.zarr.zarrjava.v3.codec.core.BytesCodec;
import dev.zarr.zarrjava.v3.codec.core.Crc32cCodec;
import dev.zarr.zarrjava.v3.codec.core.ShardingIndexedCodec;
import dev.zarr.zarrjava.v3.codec.core.TransposeCodec;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/**
 * Recognises the device-supported codec chains (zarrhip.h zh_codec_chain) and packs the
 * zh_array_meta fields the JNI shim expects.  Anything else → null (use the reference).
 */
final class DeviceChain {
    final int[] meta = new int[15]; // ndim, dtypeSize, isBool, sharded, hasTranspose, endian,
                                    // indexEndian, indexCrc32c, indexLocation, nested,
                                    // nestedIndexEndian, nestedIndexCrc32c,
                                    // nestedIndexLocation, innerCrc32c, isFloat
    // sharded: the inner chunk shape; nested: inner chunk shape followed by the leaf shape
    final long[] shape;
    final int[] chunkShape;
    int[] innerShape;
    int[] order;
    final byte[] fill;
    // byte-to-byte codecs after `bytes` that run on the host (zstd, gzip, blosc, and a crc32c
    // that is not the only one), decoded per chunk before the bytes reach the device; null
    // when the device takes the chunk bytes as stored
    BytesBytesCodec[] innerHost;

    private DeviceChain(CoreArrayMetadata m) {
        shape = m.shape.clone();
        chunkShape = m.chunkShape.clone();
        meta[0] = m.ndim();
        meta[1] = m.dataType.getByteCount();
        meta[2] = "bool".equals(m.dataType.toString().toLowerCase()) ? 1 : 0;
        // float32 / float64: the write path's all-fill test compares as == (a ±0 fill)
        String dt = m.dataType.toString().toLowerCase();
        meta[14] = "float32".equals(dt) || "float64".equals(dt) ? 1 : 0;
        fill = fillBytes(m);
    }

    static byte[] fillBytes(CoreArrayMetadata m) {
        int n = m.dataType.getByteCount();
        ByteBuffer b = ByteBuffer.allocate(8).order(ByteOrder.LITTLE_ENDIAN);
        Object f = m.parsedFillValue;
        if (f instanceof Boolean) b.put((byte) (((Boolean) f) ? 1 : 0));
        else if (f instanceof Byte) b.put((Byte) f);
        else if (f instanceof Short) b.putShort((Short) f);
        else if (f instanceof Integer) b.putInt((Integer) f);
        else if (f instanceof Long) b.putLong((Long) f);
        else if (f instanceof Float) b.putFloat((Float) f);
        else if (f instanceof Double) b.putDouble((Double) f);
        byte[] out = new byte[n];
        System.arraycopy(b.array(), 0, out, 0, n);
        return out;
    }

    private static boolean innerChain(DeviceChain d, Codec[] codecs) {
        int i = 0;
        if (i < codecs.length && codecs[i] instanceof TransposeCodec) {
            d.meta[4] = 1;
            d.order = ((TransposeCodec) codecs[i]).configuration.order.clone();
            i++;
        }
        if (i >= codecs.length || !(codecs[i] instanceof BytesCodec)) return false;
        BytesCodec bc = (BytesCodec) codecs[i];
        d.meta[5] = bc.configuration != null
                && bc.configuration.endian == BytesCodec.Endian.BIG ? 1 : 0;
        i++;
        if (i == codecs.length - 1 && codecs[i] instanceof Crc32cCodec) {  // verified on the device
            d.meta[13] = 1;
            return true;
        }
        if (i == codecs.length) return true;
        // the host decompression hand-off (north star: blosc/gzip/zstd stay on the host): the
        // remaining byte-to-byte codecs are undone per chunk with the reference's own codec
        // objects, and the device gets the raw `bytes` payload
        BytesBytesCodec[] host = new BytesBytesCodec[codecs.length - i];
        for (int k = i; k < codecs.length; k++) {
            if (!(codecs[k] instanceof BytesBytesCodec)) return false;
            host[k - i] = (BytesBytesCodec) codecs[k];
        }
        d.innerHost = host;
        return true;
    }

    /** ShardingIndexedCodec.getShardIndexSize (:176-181): 16 per inner chunk (+ 4 crc32c). */
    long indexSize() {
        long n = 1;
        for (int d = 0; d < meta[0]; d++) n *= chunkShape[d] / innerShape[d];
        return 16 * n + (meta[7] == 1 ? 4 : 0);
    }

    /** The raw `bytes` payload of one stored chunk: the host stages decoded in reverse order. */
    byte[] hostDecode(byte[] stored) throws ZarrException {
        ByteBuffer b = ByteBuffer.wrap(stored);
        for (int k = innerHost.length - 1; k >= 0; k--) b = innerHost[k].decode(b);
        byte[] out = new byte[b.remaining()];
        b.duplicate().get(out);
        return out;
    }

    /** index_codecs [bytes, crc32c?] → {endian, crc}, or null. */
    private static int[] indexChain(Codec[] ic) {
        if (ic.length < 1 || ic.length > 2 || !(ic[0] instanceof BytesCodec)) return null;
        if (ic.length == 2 && !(ic[1] instanceof Crc32cCodec)) return null;
        BytesCodec ib = (BytesCodec) ic[0];
        int be = ib.configuration != null && ib.configuration.endian == BytesCodec.Endian.BIG ? 1 : 0;
        return new int[]{be, ic.length == 2 ? 1 : 0};
    }

    /** Chain of a v3 array's codec list, or null when not device-supported. */
    static DeviceChain of(Codec[] codecs, CoreArrayMetadata m) {
        DeviceChain d = new DeviceChain(m);
        if (codecs.length == 1 && codecs[0] instanceof ShardingIndexedCodec) {
            ShardingIndexedCodec.Configuration c = ((ShardingIndexedCodec) codecs[0]).configuration;
            d.meta[3] = 1;
            d.innerShape = c.chunkShape.clone();
            if (c.codecs.length == 1 && c.codecs[0] instanceof ShardingIndexedCodec) {
                // nested sharding (ZarrPythonTests.java:177-179): one level is flattened on
                // the device; deeper nesting stays on the Java path
                ShardingIndexedCodec.Configuration nc =
                        ((ShardingIndexedCodec) c.codecs[0]).configuration;
                int n = c.chunkShape.length;
                d.innerShape = new int[2 * n];
                System.arraycopy(c.chunkShape, 0, d.innerShape, 0, n);
                System.arraycopy(nc.chunkShape, 0, d.innerShape, n, n);
                int[] nix = indexChain(nc.indexCodecs);
                if (nix == null) return null;
                d.meta[9] = 1;
                d.meta[10] = nix[0];
                d.meta[11] = nix[1];
                d.meta[12] = "start".equals(nc.indexLocation) ? 1 : 0;
                if (!innerChain(d, nc.codecs) || d.innerHost != null) return null;
            } else if (!innerChain(d, c.codecs)) {
                return null;
            }
            int[] ix = indexChain(c.indexCodecs);
            if (ix == null) return null;
            d.meta[6] = ix[0];
            d.meta[7] = ix[1];
            d.meta[8] = "start".equals(c.indexLocation) ? 1 : 0;
            return d;
        }
        return innerChain(d, codecs) ? d : null;
    }
}
