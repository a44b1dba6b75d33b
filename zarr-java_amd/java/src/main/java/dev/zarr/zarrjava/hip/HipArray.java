package dev.zarr.zarrjava.hip;

import dev.zarr.zarrjava.ZarrException;
import dev.zarr.zarrjava.store.FilesystemStore;
import dev.zarr.zarrjava.store.StoreHandle;
import dev.zarr.zarrjava.utils.IndexingUtils;
import dev.zarr.zarrjava.utils.Utils;
import dev.zarr.zarrjava.v3.Array;
import dev.zarr.zarrjava.v3.ArrayMetadata;

import javax.annotation.Nonnull;
import java.io.IOException;
import java.nio.ByteBuffer;
import java.util.stream.IntStream;

/**
 * v3.Array whose {@code read(offset, shape, parallel)} hands every chunk/shard of the
 * region to the device in ONE native call (thousands of inner chunks per launch) instead
 * of the per-shard ForkJoin loop of core.Array.read (M/core/Array.java:378-441).
 * Unsupported chains use {@code super.read}.
 *
 * Over a FilesystemStore (no host byte-to-byte stages; ZH_DEVICES: one slab per device) the
 * chunk files' paths
 * (StoreHandle.toPath(), M/store/StoreHandle.java:100-105) go to the library, which does the
 * store reads itself (arrayReadFiles).  Otherwise the store I/O keeps the reference's shape and
 * parallelism (the chunk loop runs as a parallel stream, M/core/Array.java:403-407): a whole
 * shard is one read; a sub-shard part is its stored index plus the ranges it references
 * (ShardPieces, StoreHandleDataProvider semantics).  The index is checked on the device.
 */
public class HipArray extends Array {
    private final DeviceChain chain;

    protected HipArray(StoreHandle storeHandle, ArrayMetadata metadata) throws ZarrException {
        super(storeHandle, metadata);
        chain = ZarrHip.available() ? DeviceChain.of(metadata.codecs, metadata.coreArrayMetadata)
                : null;
    }

    public static HipArray open(StoreHandle storeHandle) throws IOException, ZarrException {
        Array a = Array.open(storeHandle);
        return new HipArray(storeHandle, a.metadata());
    }

    @Nonnull
    @Override
    public ucar.ma2.Array read(final long[] offset, final long[] shape, final boolean parallel)
            throws ZarrException {
        if (chain == null) return super.read(offset, shape, parallel);
        ArrayMetadata md = metadata();
        // core.Array.read's argument checks, same order and messages (M/core/Array.java:380-390)
        if (offset.length != md.ndim()) {
            throw new IllegalArgumentException("'offset' needs to have rank '" + md.ndim() + "'.");
        }
        if (shape.length != md.ndim()) {
            throw new IllegalArgumentException("'shape' needs to have rank '" + md.ndim() + "'.");
        }
        for (int d = 0; d < md.ndim(); d++) {
            if (offset[d] < 0 || offset[d] + shape[d] > md.shape[d]) {
                throw new ZarrException("Requested data is outside of the array's domain.");
            }
        }
        final int[] cs = md.chunkShape();
        final long[][] coords = IndexingUtils.computeChunkCoords(md.shape, cs, offset, shape);
        final boolean sharded = chain.meta[3] == 1;
        long[] ctxs = ZarrHip.ctxs();
        if (storeHandle.store instanceof FilesystemStore && chain.innerHost == null) {
            // the library reads the chunk files itself (FilesystemStore.exists / get semantics,
            // M/store/FilesystemStore.java:43-102): pread into its page-locked ring, overlapped
            // with the device work; nothing of the chunks enters the Java heap
            String[] paths = new String[coords.length];
            for (int i = 0; i < coords.length; i++) {
                paths[i] = storeHandle.resolve(md.chunkKeyEncoding().encodeChunkKey(coords[i]))
                        .toPath().toString();
            }
            ucar.ma2.Array out = ucar.ma2.Array.factory(md.dataType().getMA2DataType(),
                    Utils.toIntArray(shape));
            int st = ZarrHip.arrayReadFiles(ctxs, chain.meta, chain.shape, chain.chunkShape,
                    chain.innerShape, chain.order, chain.fill,
                    ZarrHip.storeRoot(storeHandle.store), storeHandle.store.toString(), paths,
                    offset, shape, out.getStorage());
            return st == 0 ? out : super.read(offset, shape, parallel);
        }
        final ShardPieces[] shards = new ShardPieces[coords.length];
        final byte[][] chunks = new byte[coords.length][];
        IntStream loop = IntStream.range(0, coords.length);
        try {
            (parallel ? loop.parallel() : loop).forEach(i -> {
                StoreHandle h = storeHandle.resolve(md.chunkKeyEncoding().encodeChunkKey(coords[i]));
                try {
                    if (sharded) {
                        long[] lo = new long[cs.length], hi = new long[cs.length];
                        for (int d = 0; d < cs.length; d++) {
                            long c0 = coords[i][d] * cs[d];
                            lo[d] = Math.max(offset[d], c0) - c0;
                            hi[d] = Math.min(offset[d] + shape[d], c0 + cs[d]) - c0;
                        }
                        shards[i] = ShardPieces.isWhole(chain, lo, hi) ? ShardPieces.whole(h)
                                : ShardPieces.part(h, chain, lo, hi);
                        return;
                    }
                    ByteBuffer b = h.read();
                    if (b != null) {
                        chunks[i] = ShardPieces.bytes(b);
                        // unsharded chain with host stages (e.g. [bytes, zstd]): raw payload
                        if (chain.innerHost != null) chunks[i] = chain.hostDecode(chunks[i]);
                    }
                } catch (ZarrException e) {
                    throw new RuntimeException(e);
                }
            });
        } catch (RuntimeException e) {
            if (e.getCause() instanceof ZarrException) throw (ZarrException) e.getCause();
            throw e;
        }
        ucar.ma2.Array out = ucar.ma2.Array.factory(md.dataType().getMA2DataType(),
                Utils.toIntArray(shape));
        int st;
        if (sharded) {
            st = ZarrHip.arrayReadPieces(ctxs, chain.meta, chain.shape, chain.chunkShape,
                    chain.innerShape, chain.order, chain.fill, ZarrHip.indexes(shards),
                    ZarrHip.sizes(shards), ZarrHip.pieceOffsets(shards),
                    ZarrHip.pieceLens(shards), ZarrHip.pieceData(shards), offset, shape,
                    out.getStorage());
        } else {
            st = ctxs.length > 1
                    ? ZarrHip.arrayReadMulti(ctxs, chain.meta, chain.shape, chain.chunkShape,
                            chain.innerShape, chain.order, chain.fill, chunks, offset, shape,
                            out.getStorage())
                    : ZarrHip.arrayRead(ctxs[0], chain.meta, chain.shape, chain.chunkShape,
                            chain.innerShape, chain.order, chain.fill, chunks, offset, shape,
                            out.getStorage());
        }
        return st == 0 ? out : super.read(offset, shape, parallel);
    }

    /**
     * core.Array.write (M/core/Array.java:83-133) + writeChunk (:143-156) in one device call
     * when the region covers whole chunks (clipped only by the array boundary): every chunk is
     * encoded on the device (ShardingIndexedCodec.encode incl. the all-fill elision) and then
     * stored, or deleted when it is all fill_value.  Regions that cut chunks need the
     * read-modify-write of core.Array.write and take {@code super.write}.
     */
    @Override
    public void write(long[] offset, ucar.ma2.Array array, boolean parallel) {
        ArrayMetadata md = metadata();
        // zh_array_write_host emits raw `bytes` payloads only: chains with host byte-to-byte
        // stages (zstd, gzip, blosc, a non-final crc32c) keep the reference's encode, and the
        // region's element type must be the array's (its bytes are copied as dtype elements)
        if (chain == null || chain.innerHost != null || offset.length != md.ndim()
                || array.getRank() != md.ndim()
                || array.getDataType().getSize() != md.dataType().getByteCount()
                || array.getDataType().isFloatingPoint()
                    != md.dataType().getMA2DataType().isFloatingPoint()) {
            super.write(offset, array, parallel);
            return;
        }
        long[] shape = Utils.toLongArray(array.getShape());
        int[] cs = md.chunkShape();
        for (int d = 0; d < md.ndim(); d++) {
            long end = offset[d] + shape[d];
            if (offset[d] % cs[d] != 0 || (end % cs[d] != 0 && end != md.shape[d])) {
                super.write(offset, array, parallel);
                return;
            }
        }
        if (storeHandle.store instanceof FilesystemStore && md.parsedFillValue() != null) {
            // the library encodes and writes (or deletes) the chunk files itself
            // (FilesystemStore.set / delete semantics, M/store/FilesystemStore.java:105-142)
            long[][] coords = IndexingUtils.computeChunkCoords(md.shape, cs, offset, shape);
            String[] paths = new String[coords.length];
            for (int i = 0; i < coords.length; i++) {
                paths[i] = storeHandle.resolve(md.chunkKeyEncoding().encodeChunkKey(coords[i]))
                        .toPath().toString();
            }
            if (ZarrHip.arrayWriteFiles(ZarrHip.ctx(), chain.meta, chain.shape, chain.chunkShape,
                    chain.innerShape, chain.order, chain.fill, offset, shape,
                    array.copyTo1DJavaArray(), ZarrHip.storeRoot(storeHandle.store),
                    storeHandle.store.toString(), paths) == 0) {
                return;
            }
        }
        byte[][] enc = ZarrHip.arrayWrite(ZarrHip.ctx(), chain.meta, chain.shape,
                chain.chunkShape, chain.innerShape, chain.order, chain.fill, offset, shape,
                array.copyTo1DJavaArray());
        if (enc == null) {
            super.write(offset, array, parallel);
            return;
        }
        long[][] coords = IndexingUtils.computeChunkCoords(md.shape, cs, offset, shape);
        for (int i = 0; i < coords.length; i++) {
            StoreHandle h = storeHandle.resolve(md.chunkKeyEncoding().encodeChunkKey(coords[i]));
            if (enc[i] == null) {
                h.delete();
            } else {
                h.set(ByteBuffer.wrap(enc[i]));
            }
        }
    }
}
