package dev.zarr.zarrjava.hip;

import dev.zarr.zarrjava.ZarrException;
import dev.zarr.zarrjava.store.StoreHandle;
import dev.zarr.zarrjava.utils.IndexingUtils;
import dev.zarr.zarrjava.utils.Utils;
import dev.zarr.zarrjava.v3.Array;
import dev.zarr.zarrjava.v3.ArrayMetadata;

import javax.annotation.Nonnull;
import java.io.IOException;
import java.nio.ByteBuffer;

/**
 * v3.Array whose {@code read(offset, shape, parallel)} hands every chunk/shard of the
 * region to the device in ONE native call (thousands of inner chunks per launch) instead
 * of the per-shard ForkJoin loop of core.Array.read (M/core/Array.java:378-441).
 * Unsupported chains use {@code super.read}.
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
        for (int d = 0; d < md.ndim(); d++) {
            if (offset[d] < 0 || offset[d] + shape[d] > md.shape[d]) {
                throw new ZarrException("Requested data is outside of the array's domain.");
            }
        }
        long[][] coords = IndexingUtils.computeChunkCoords(md.shape, md.chunkShape(), offset, shape);
        byte[][] chunks = new byte[coords.length][];
        for (int i = 0; i < coords.length; i++) {
            StoreHandle h = storeHandle.resolve(md.chunkKeyEncoding().encodeChunkKey(coords[i]));
            ByteBuffer b = h.read();
            if (b != null) {
                chunks[i] = new byte[b.remaining()];
                b.duplicate().get(chunks[i]);
            }
        }
        ucar.ma2.Array out = ucar.ma2.Array.factory(md.dataType().getMA2DataType(),
                Utils.toIntArray(shape));
        long[] ctxs = ZarrHip.ctxs();
        int st = ctxs.length > 1
                ? ZarrHip.arrayReadMulti(ctxs, chain.meta, chain.shape, chain.chunkShape,
                        chain.innerShape, chain.order, chain.fill, chunks, offset, shape,
                        out.getStorage())
                : ZarrHip.arrayRead(ctxs[0], chain.meta, chain.shape, chain.chunkShape,
                        chain.innerShape, chain.order, chain.fill, chunks, offset, shape,
                        out.getStorage());
        return st == 0 ? out : super.read(offset, shape, parallel);
    }
}
