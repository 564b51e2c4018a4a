package com.backblaze.erasure.ecx;

import java.nio.ByteBuffer;

/**
 * ReedSolomon.encodeParity / decodeMissing (ReedSolomon.java:94-108, :189-286) over many
 * stripes kept in the engine's blocked layout in host memory (ecx_rs_*_blocked_batch_host,
 * DESIGN.md section 4.6): a direct ByteBuffer of nstripes * (dataShards + parityShards) *
 * byteCount bytes, each stripe's full blocks block-major ([block][shard][block bytes]) and the
 * tails of all stripes after the full blocks of all stripes ([stripe][shard][tail]).  A caller
 * that keeps its stripes blocked end to end feeds the GPU the layout its kernels run fastest on
 * (RS(17,3) on 200,000-B shards: 0.768 of HBM against 0.70 on back-to-back shards), with no
 * packing pass; {@link Ecx#blockedLayout} gives the block size to lay the stripes out with.
 */
public final class EcxBlockedStripes {
    private long rs;  // 0 once closed
    private final int dataShards;
    private final int parityShards;

    /** The codec of ReedSolomon.create(dataShards, parityShards). */
    public EcxBlockedStripes(int dataShards, int parityShards) {
        this.rs = Ecx.createReedSolomon(dataShards, parityShards);
        this.dataShards = dataShards;
        this.parityShards = parityShards;
    }

    /** {block bytes, full blocks per shard, tail bytes} of the recommended layout (Ecx.blockedLayout). */
    public long[] layout(long byteCount) {
        return Ecx.blockedLayout(dataShards, parityShards, byteCount);
    }

    /**
     * encodeParity over every stripe, in place: the parity shards' blocks and tails are
     * overwritten.  blockBytes 0 = the recommended block ({@link #layout}).
     */
    public void encodeParity(ByteBuffer stripes, long nstripes, long byteCount, long blockBytes) {
        checkExtent(stripes, nstripes, byteCount);
        Ecx.check(EcxNative.rsEncodeParityBlockedBatchHostBuffer(handle(), stripes, nstripes, byteCount, blockBytes));
    }

    /**
     * decodeMissing over every stripe, in place: the shards with shardPresent[i] == false are
     * rebuilt from the first dataShards present ones, as ReedSolomon.decodeMissing does.
     */
    public void decodeMissing(ByteBuffer stripes, boolean[] shardPresent, long nstripes, long byteCount,
                              long blockBytes) {
        byte[] flags = flags(shardPresent);
        checkExtent(stripes, nstripes, byteCount);
        Ecx.check(EcxNative.rsDecodeMissingBlockedBatchHostBuffer(handle(), flags, stripes, nstripes, byteCount,
                blockBytes));
    }

    /**
     * encodeParity split over several GPUs of this JVM: contiguous stripe ranges, one worker thread
     * and stream set per entry of {@code devices} (ecx_rs_encode_parity_blocked_batch_host_devices).
     */
    public void encodeParity(ByteBuffer stripes, long nstripes, long byteCount, long blockBytes, int[] devices) {
        checkExtent(stripes, nstripes, byteCount);
        Ecx.check(EcxNative.rsEncodeParityBlockedBatchHostDevicesBuffer(handle(), stripes, nstripes, byteCount,
                blockBytes, devices, devices == null ? 0 : devices.length));
    }

    /** decodeMissing split over several GPUs of this JVM (ecx_rs_decode_missing_blocked_batch_host_devices). */
    public void decodeMissing(ByteBuffer stripes, boolean[] shardPresent, long nstripes, long byteCount,
                              long blockBytes, int[] devices) {
        byte[] flags = flags(shardPresent);
        checkExtent(stripes, nstripes, byteCount);
        Ecx.check(EcxNative.rsDecodeMissingBlockedBatchHostDevicesBuffer(handle(), flags, stripes, nstripes,
                byteCount, blockBytes, devices, devices == null ? 0 : devices.length));
    }

    private byte[] flags(boolean[] shardPresent) {
        int n = dataShards + parityShards;
        if (shardPresent == null) {
            throw new NullPointerException("shardPresent");
        }
        if (shardPresent.length != n) {
            throw new IllegalArgumentException("wrong number of shardPresent flags: " + shardPresent.length);
        }
        byte[] flags = new byte[n];
        for (int i = 0; i < n; i++) {
            flags[i] = (byte) (shardPresent[i] ? 1 : 0);
        }
        return flags;
    }

    // The forwarder checks the same extent from the buffer's capacity; this gives the message.
    private void checkExtent(ByteBuffer stripes, long nstripes, long byteCount) {
        if (nstripes <= 0 || byteCount <= 0 || stripes == null) {
            return;
        }
        long need = nstripes * (dataShards + parityShards) * byteCount;
        if (need > stripes.capacity()) {
            throw new ArrayIndexOutOfBoundsException("the stripes need " + need + " bytes, the buffer holds "
                    + stripes.capacity());
        }
    }

    private long handle() {
        if (rs == 0) {
            throw new IllegalStateException("EcxBlockedStripes is closed");
        }
        return rs;
    }

    /** Releases this wrapper's reference to the shared native codec; idempotent (see EcxPartialSums). */
    public synchronized void close() {
        if (rs == 0) {
            return;
        }
        long h = rs;
        rs = 0;
        EcxNative.rsDestroy(h);
    }
}
