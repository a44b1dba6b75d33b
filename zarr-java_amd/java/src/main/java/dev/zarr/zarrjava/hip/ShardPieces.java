package dev.zarr.zarrjava.hip;

import dev.zarr.zarrjava.ZarrException;
import dev.zarr.zarrjava.store.StoreHandle;

import java.nio.ByteBuffer;

/**
 * The store I/O of a shard read, and nothing else: StoreHandleDataProvider's reads
 * (M/v3/codec/core/ShardingIndexedCodec.java:190-230, 333-357).  For a sub-shard part: one
 * prefix/suffix read of the stored index, zh_shard_ranges (via JNI) for the byte ranges the part
 * references, one store read per range.  For a whole shard: one read.  The stored index is
 * handed to the device unchanged, where its crc32c (Crc32cCodec.java:24-48) and its entries are
 * checked; nothing here parses or trusts it (with host stages or an unknown shard size the
 * crc32c is checked on the host first, see part()).  No shard is ever assembled on the heap, so a part
 * whose referenced payload exceeds 2^31 bytes reads like any other (each range is at most
 * 64 MiB; one inner chunk with host stages).
 *
 * With host byte-to-byte stages in the inner chain (DeviceChain.innerHost: zstd, gzip, blosc)
 * every inner chunk is read and decoded on its own: its piece holds the raw payload.
 */
final class ShardPieces {
    /** Longest run of adjacent inner chunks fetched by one store read. */
    static final long MAX_RUN = 64L << 20;

    /** The stored index as read (null: the shard is whole in piece 0). */
    final byte[] index;
    /** StoreHandle.getSize(), or -1 when the store cannot tell. */
    final long shardSize;
    /** Per piece: shard byte offset, stored length, bytes (raw, or decoded by the host stages). */
    final long[] offsets;
    final long[] storedLens;
    final byte[][] data;

    private ShardPieces(byte[] index, long shardSize, long[] offsets, long[] storedLens,
                        byte[][] data) {
        this.index = index;
        this.shardSize = shardSize;
        this.offsets = offsets;
        this.storedLens = storedLens;
        this.data = data;
    }

    /** The bytes behind a store read, without a copy when it is a whole heap array. */
    static byte[] bytes(ByteBuffer b) {
        if (b.hasArray() && b.arrayOffset() == 0 && b.position() == 0
                && b.remaining() == b.array().length) {
            return b.array();
        }
        byte[] out = new byte[b.remaining()];
        b.duplicate().get(out);
        return out;
    }

    /** The whole shard as one piece at offset 0, or null when the key is missing. */
    static ShardPieces whole(StoreHandle h) {
        ByteBuffer b = h.read();
        if (b == null) return null;
        byte[] all = bytes(b);
        return new ShardPieces(null, all.length, new long[]{0}, new long[]{all.length},
                new byte[][]{all});
    }

    /**
     * The part [partLo, partHi) (shard-local element coordinates) of the shard at {@code h}:
     * its stored index and the ranges it references, or null when the shard is missing.
     */
    static ShardPieces part(StoreHandle h, DeviceChain chain, long[] partLo, long[] partHi)
            throws ZarrException {
        final boolean start = chain.meta[8] == 1;
        final long isz = chain.indexSize();
        if (!h.exists()) return null;
        ByteBuffer ib = start ? h.read(0, isz) : h.read(-isz);
        if (ib == null) return null;
        byte[] index = bytes(ib);
        // StoreHandle.getSize() is -1 when the store cannot tell (an HTTP HEAD without
        // Content-Length, a failed HEAD): the ranges are then bounded by the reads themselves.
        // A FilesystemStore range read past the end of the file returns zeros
        // (FilesystemStore.get(keys, start, end), M/store/FilesystemStore.java:84-102), so no
        // entry is out of its reach by offset: the size bounds nothing there either.
        long size = h.store instanceof dev.zarr.zarrjava.store.FilesystemStore ? -1 : h.getSize();
        if (size < 0) size = -1;
        if (index.length < isz) {  // the device reports "Shard ... is smaller than its index"
            return new ShardPieces(index, size, new long[0], new long[0], new byte[0][]);
        }
        final boolean host = chain.innerHost != null;
        // The index decides host work before the device sees it when the ranges are decoded
        // on the host (innerHost) or the shard size is unknown (a corrupt entry could ask for a
        // 2^31-byte read): then its crc32c is checked here first, as the reference checks it
        // before any range read (ShardingIndexedCodec.java:205); a mismatch throws the
        // reference's ZarrException.  Otherwise the device checks it.
        final boolean check = chain.meta[7] == 1 && (host || size < 0);
        long[] rs = ZarrHip.shardRanges(chain.meta, chain.shape, chain.chunkShape,
                chain.innerShape, chain.order, chain.fill, index, size, partLo, partHi,
                host ? 0 : MAX_RUN, check);
        int n = rs.length / 2, k = 0;
        long[] offs = new long[n], lens = new long[n];
        byte[][] data = new byte[n][];
        for (int r = 0; r < n; r++) {
            long off = rs[2 * r], nb = rs[2 * r + 1];
            ByteBuffer blob = h.read(off, off + nb);
            if (blob == null || blob.remaining() < nb) {
                // the store could not deliver the range: the device reports the reference's
                // "Could not load byte data for chunk [...]" for the entries it held
                continue;
            }
            byte[] b = bytes(blob);
            offs[k] = off;
            lens[k] = nb;
            data[k] = host ? chain.hostDecode(b) : b;
            k++;
        }
        if (k < n) {
            offs = java.util.Arrays.copyOf(offs, k);
            lens = java.util.Arrays.copyOf(lens, k);
            data = java.util.Arrays.copyOf(data, k);
        }
        return new ShardPieces(index, size, offs, lens, data);
    }

    /**
     * True when [partLo, partHi) is the whole shard and its stored bytes can go to the device
     * as they are (no host stages to undo).
     */
    static boolean isWhole(DeviceChain chain, long[] partLo, long[] partHi) {
        if (chain.innerHost != null) return false;
        for (int d = 0; d < chain.meta[0]; d++) {
            if (partLo[d] != 0 || partHi[d] != chain.chunkShape[d]) return false;
        }
        return true;
    }
}
