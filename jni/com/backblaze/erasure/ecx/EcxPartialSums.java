package com.backblaze.erasure.ecx;

/**
 * The repair-pipelining partial sums of ReedSolomon (encodeParitySingle,
 * ReedSolomon.java:110-118; decodeMissingSingle, :288-333), which the reference runs
 * through InputOutputByteTableCodingLoopSingle directly rather than the injected
 * CodingLoop, on libecx.so.  Drop-in sites: NodeHelper.kt:89 (LRC chain),
 * ClayCodeNode.kt:182-186 and :225-228 (Clay chain).
 */
public final class EcxPartialSums {
    private long rs;  // 0 once closed
    private final int dataShards;

    /** The codec of ReedSolomon.create(dataShards, parityShards). */
    public EcxPartialSums(int dataShards, int parityShards) {
        this.rs = Ecx.createReedSolomon(dataShards, parityShards);
        this.dataShards = dataShards;
    }

    /** ReedSolomon.encodeParitySingle: output ^= parityRows[outputIndex][inputIndex] * shard. */
    public void encodeParitySingle(byte[] shard, byte[] output, int inputIndex, int outputIndex, int offset,
                                   int byteCount) {
        Ecx.check(EcxNative.rsEncodeParitySingle(handle(), shard, output, inputIndex, outputIndex, offset, byteCount));
    }

    /**
     * NodeHelper.kt:86-97 at block granularity: the reference calls encodeParitySingle
     * once per 34-byte word (PipelineUtil.kt:10-11, 1024 calls per 34,816-byte block)
     * and forwards each word.  The partial sum is byte-wise, so one call over the whole
     * block gives every word's partial sum at once; the node then streams the words
     * from {@code output} (each word's bytes are its own range of the block).
     */
    public void encodeParitySingleBlock(byte[] block, byte[] output, int inputIndex, int outputIndex) {
        encodeParitySingle(block, output, inputIndex, outputIndex, 0, block.length);
    }

    /**
     * ReedSolomon.decodeMissingSingle: every missing data shard's share of this helper,
     * outputs[j] (=, or ^= unless isFirst) D^-1[j][index] * shard, written into the
     * caller's arrays (the reference allocates fresh ones when isFirst).  No missing
     * data shard: NullPointerException, as the reference (SURVEY.md A.2, B3).
     */
    public void decodeMissingSingle(byte[] shard, int shardIndex, int index, boolean[] shardPresent,
                                    byte[][] outputs, int offset, int byteCount, boolean isFirst) {
        if (isFirst && shardIndex < dataShards) {
            for (int j = 0; j < outputs.length; j++) {
                if (outputs[j] == null) {
                    outputs[j] = new byte[offset + byteCount];
                }
            }
        }
        Ecx.check(EcxNative.rsDecodeMissingSingle(handle(), shard, shardIndex, index, Ecx.flags(shardPresent), outputs,
                null, outputs.length, offset, byteCount, isFirst ? 1 : 0));
    }

    private long handle() {
        if (rs == 0) {
            throw new IllegalStateException("EcxPartialSums is closed");
        }
        return rs;
    }

    /**
     * Releases this wrapper's reference to the native codec.  Idempotent: the codec is
     * shared by every wrapper of the same (k, m) (ecx_rs_create), so a second release would
     * drop another wrapper's reference; later calls on this wrapper throw IllegalStateException.
     */
    public synchronized void close() {
        if (rs == 0) {
            return;
        }
        long h = rs;
        rs = 0;
        EcxNative.rsDestroy(h);
    }
}
