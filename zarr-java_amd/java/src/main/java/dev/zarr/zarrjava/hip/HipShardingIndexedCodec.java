package dev.zarr.zarrjava.hip;

import com.fasterxml.jackson.annotation.JsonCreator;
import com.fasterxml.jackson.annotation.JsonProperty;
import dev.zarr.zarrjava.ZarrException;
import dev.zarr.zarrjava.core.ArrayMetadata.CoreArrayMetadata;
import dev.zarr.zarrjava.store.FilesystemStore;
import dev.zarr.zarrjava.store.StoreHandle;
import dev.zarr.zarrjava.v3.codec.Codec;
import dev.zarr.zarrjava.v3.codec.core.ShardingIndexedCodec;
import ucar.ma2.Array;

import javax.annotation.Nonnull;
import java.nio.ByteBuffer;
import java.util.Arrays;

/**
 * Drop-in `sharding_indexed` codec whose decode runs on the MI355X.  Registered with
 * {@code CodecRegistry.addType("sharding_indexed", HipShardingIndexedCodec.class)}; it
 * extends the reference codec so `instanceof ShardingIndexedCodec` discovery
 * (v3/ArrayMetadata.java) and CodecPipeline.supportsPartialDecode keep working, and falls
 * back to {@code super} for chains the device does not run.
 */
public class HipShardingIndexedCodec extends ShardingIndexedCodec {
    private DeviceChain chain;

    @JsonCreator(mode = JsonCreator.Mode.PROPERTIES)
    public HipShardingIndexedCodec(
            @Nonnull @JsonProperty(value = "configuration", required = true)
            Configuration configuration) throws ZarrException {
        super(configuration);
    }

    @Override
    public void setCoreArrayMetadata(CoreArrayMetadata arrayMetadata) throws ZarrException {
        super.setCoreArrayMetadata(arrayMetadata);
        chain = ZarrHip.available() ? DeviceChain.of(new Codec[]{this}, arrayMetadata) : null;
    }

    private Array device(byte[] shard, long[] offset, int[] shape) throws ZarrException {
        Array out = Array.factory(arrayMetadata.dataType.getMA2DataType(), shape);
        int st = ZarrHip.shardDecodePartial(ZarrHip.codecCtx(), chain.meta, chain.shape,
                chain.chunkShape, chain.innerShape, chain.order, chain.fill, shard, offset, shape,
                out.getStorage());
        return st == 0 ? out : null;
    }

    @Override
    public Array decode(ByteBuffer shardBytes) throws ZarrException {
        if (chain != null && chain.innerHost == null) {  // host stages: decodePartial stages them
            byte[] b = new byte[shardBytes.remaining()];
            shardBytes.duplicate().get(b);
            Array a = device(b, new long[arrayMetadata.ndim()], arrayMetadata.chunkShape);
            if (a != null) return a;
        }
        return super.decode(shardBytes);
    }

    @Override
    public Array decodePartial(StoreHandle chunkHandle, long[] offset, int[] shape)
            throws ZarrException {
        if (chain != null && chain.innerHost == null
                && chunkHandle.store instanceof FilesystemStore) {
            // the library reads the shard file itself (zh_array_read_files over the shard viewed
            // as a one-chunk array): the stored index, then the referenced ranges
            java.nio.file.Path path = chunkHandle.toPath();
            if (java.nio.file.Files.isRegularFile(path)) {
                long[] shardShape = new long[shape.length], part = new long[shape.length];
                for (int d = 0; d < shape.length; d++) {
                    shardShape[d] = chain.chunkShape[d];
                    part[d] = shape[d];
                }
                Array out = Array.factory(arrayMetadata.dataType.getMA2DataType(), shape);
                int st = ZarrHip.arrayReadFiles(new long[]{ZarrHip.codecCtx()}, chain.meta,
                        shardShape,
                        chain.chunkShape, chain.innerShape, chain.order, chain.fill,
                        ZarrHip.storeRoot(chunkHandle.store), chunkHandle.store.toString(),
                        new String[]{path.toString()}, offset, part, out.getStorage());
                if (st == 0) return out;
            }
        }
        if (chain != null) {
            long[] hi = new long[offset.length];
            for (int d = 0; d < offset.length; d++) hi[d] = offset[d] + shape[d];
            // the whole shard in one read, or its stored index + the referenced ranges
            // (StoreHandleDataProvider, ShardingIndexedCodec.java:245-255, 333-357)
            ShardPieces p = ShardPieces.isWhole(chain, offset, hi) ? ShardPieces.whole(chunkHandle)
                    : ShardPieces.part(chunkHandle, chain, offset, hi);
            if (p == null) {
                return Arrays.equals(shape, arrayMetadata.chunkShape)
                        ? arrayMetadata.allocateFillValueChunk()
                        : super.decodePartial(chunkHandle, offset, shape);
            }
            Array out = Array.factory(arrayMetadata.dataType.getMA2DataType(), shape);
            int st = ZarrHip.shardDecodePieces(ZarrHip.codecCtx(), chain.meta, chain.shape,
                    chain.chunkShape, chain.innerShape, chain.order, chain.fill, p.index,
                    p.shardSize, p.offsets, p.storedLens, p.data, offset, shape,
                    out.getStorage());
            if (st == 0) return out;
        }
        return super.decodePartial(chunkHandle, offset, shape);
    }
}
