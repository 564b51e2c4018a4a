package com.backblaze.erasure.ecx;

import java.nio.ByteBuffer;

/**
 * ReedSolomon.isParityCorrect (ReedSolomon.java:129-178) over many stripes at once, the
 * "Check" half of ReedSolomonBenchmark (:73-87,126-149), on libecx.so: the stripes sit in a
 * direct ByteBuffer (stripe s's shard i at s * stripeStride + i * shardStride), every stripe's
 * shards cross PCIe once through the read-only check kernel, and one verdict byte per stripe
 * comes back (1 = the parity is correct over [firstByte, firstByte + byteCount)).
 */
public final class EcxParityCheck {
    private long rs;  // 0 once closed
    private final int shardCount;

    /** The codec of ReedSolomon.create(dataShards, parityShards). */
    public EcxParityCheck(int dataShards, int parityShards) {
        this.rs = Ecx.createReedSolomon(dataShards, parityShards);
        this.shardCount = dataShards + parityShards;
    }

    /** verdict.get(s) == 1 iff stripe s passes isParityCorrect(shards of s, firstByte, byteCount). */
    public void isParityCorrectBatch(ByteBuffer stripes, long stripeStride, long shardStride, long nstripes,
                                     long firstByte, long byteCount, ByteBuffer verdict) {
        checkExtent(stripes, stripeStride, shardStride, nstripes, firstByte, byteCount, verdict);
        Ecx.check(EcxNative.rsIsParityCorrectBatchHostBuffer(handle(), stripes, stripeStride, shardStride, nstripes,
                firstByte, byteCount, verdict));
    }

    /**
     * The same over several GPUs of this JVM: contiguous stripe ranges, one worker thread and
     * stream set per entry of {@code devices} (ecx_rs_is_parity_correct_batch_host_devices).
     */
    public void isParityCorrectBatch(ByteBuffer stripes, long stripeStride, long shardStride, long nstripes,
                                     long firstByte, long byteCount, ByteBuffer verdict, int[] devices) {
        checkExtent(stripes, stripeStride, shardStride, nstripes, firstByte, byteCount, verdict);
        Ecx.check(EcxNative.rsIsParityCorrectBatchHostDevicesBuffer(handle(), stripes, stripeStride, shardStride,
                nstripes, firstByte, byteCount, verdict, devices, devices == null ? 0 : devices.length));
    }

    // The forwarder checks the same extents from the buffers' capacities; this gives the message.
    private void checkExtent(ByteBuffer stripes, long stripeStride, long shardStride, long nstripes, long firstByte,
                             long byteCount, ByteBuffer verdict) {
        if (nstripes <= 0 || byteCount <= 0 || stripes == null || verdict == null) {
            return;
        }
        long need = (nstripes - 1) * stripeStride + (long) (shardCount - 1) * shardStride + firstByte + byteCount;
        if (need > stripes.capacity()) {
            throw new ArrayIndexOutOfBoundsException("the stripes need " + need + " bytes, the buffer holds "
                    + stripes.capacity());
        }
        if (nstripes > verdict.capacity()) {
            throw new ArrayIndexOutOfBoundsException("the verdicts need " + nstripes + " bytes, the buffer holds "
                    + verdict.capacity());
        }
    }

    private long handle() {
        if (rs == 0) {
            throw new IllegalStateException("EcxParityCheck is closed");
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
