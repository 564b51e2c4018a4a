package com.backblaze.erasure.ecx;

import java.nio.ByteBuffer;

/**
 * Status codes of libecx.so (include/ecx.h:40-50) mapped back onto the exceptions the
 * reference throws for the same conditions, with the library's thread-local message.
 */
public final class Ecx {
    public static final int OK = 0;
    public static final int E_ILLEGAL_ARGUMENT = -1; // IllegalArgumentException (sizes, offsets, counts)
    public static final int E_NOT_ENOUGH_SHARDS = -2; // "Not enough shards present", ReedSolomon.java:211-213
    public static final int E_SINGULAR = -3;          // "Matrix is singular", Matrix.java:311-313
    public static final int E_TOO_MANY_SHARDS = -4;   // "too many shards - max is 256", ReedSolomon.java:48-50
    public static final int E_INDEX = -5;             // ArrayIndexOutOfBoundsException (Clay (k+m)%m != 0)
    public static final int E_NULL = -6;              // NullPointerException (decodeMissingSingle, bug B3)
    public static final int E_NOMEM = -7;             // host or device allocation failed
    public static final int E_DEVICE = -10;           // no HIP device / HIP runtime error

    private Ecx() {
    }

    /** Returns {@code status} if it is not an error, else throws the reference's exception. */
    public static int check(int status) {
        if (status >= 0) {
            return status;
        }
        String detail = EcxNative.lastError();
        String msg = EcxNative.statusString(status) + (detail == null || detail.isEmpty() ? "" : ": " + detail);
        switch (status) {
            case E_ILLEGAL_ARGUMENT:
            case E_NOT_ENOUGH_SHARDS:
            case E_SINGULAR:
            case E_TOO_MANY_SHARDS:
                throw new IllegalArgumentException(msg);
            case E_INDEX:
                throw new ArrayIndexOutOfBoundsException(msg);
            case E_NULL:
                throw new NullPointerException(msg);
            case E_NOMEM:
                throw new OutOfMemoryError(msg);
            default:
                throw new IllegalStateException(msg);
        }
    }

    /** Flattens row-major coefficient rows (the CodingLoop matrixRows argument). */
    public static byte[] flatten(byte[][] rows, int rowCount, int rowLength) {
        byte[] flat = new byte[rowCount * rowLength];
        for (int r = 0; r < rowCount; r++) {
            System.arraycopy(rows[r], 0, flat, r * rowLength, rowLength);
        }
        return flat;
    }

    /** boolean[] shard-present flags as the byte flags the C ABI takes. */
    public static byte[] flags(boolean[] present) {
        byte[] f = new byte[present.length];
        for (int i = 0; i < present.length; i++) {
            f[i] = (byte) (present[i] ? 1 : 0);
        }
        return f;
    }

    /**
     * A direct ByteBuffer of exactly {@code nbytes} over page-locked host memory
     * (ecx_host_alloc), for the host-batch calls to run at the PCIe rate.  Its capacity is the
     * allocation's size, so the capacity-checked host-batch natives bound every access to it.
     * Release it with {@link #freePinned}.
     */
    public static ByteBuffer allocatePinned(long nbytes) {
        if (nbytes < 0) {
            throw new IllegalArgumentException("negative size");
        }
        long[] p = new long[1];
        check(EcxNative.hostAlloc(nbytes, p));
        return EcxNative.wrapAddress(p[0], nbytes);
    }

    /** Frees a buffer from {@link #allocatePinned}; the buffer must not be used afterwards. */
    public static void freePinned(ByteBuffer buffer) {
        check(EcxNative.hostFree(EcxNative.directAddress(buffer)));
    }

    /**
     * The shard pitch to give a pool of RS(dataShards, parityShards) stripes kept as
     * [stripe][shard][pitch] (ecx_rs_recommended_pitch, DESIGN.md section 4.6): the smallest odd
     * multiple of 4 KiB at or above {@code byteCount}, e.g. to size an {@link #allocatePinned}
     * pool as nstripes * (dataShards + parityShards) * pitch bytes.
     */
    public static long recommendedPitch(int dataShards, int parityShards, long byteCount) {
        long[] p = new long[1];
        check(EcxNative.rsRecommendedPitch(dataShards, parityShards, byteCount, p));
        return p[0];
    }

    /**
     * The engine's blocked layout for RS(dataShards, parityShards) stripes of byteCount-byte
     * shards (ecx_rs_blocked_layout): {block bytes, full blocks per shard, tail bytes}.  A stripe's
     * full blocks lie block-major, [block][shard][block bytes]; the tails of all stripes follow the
     * full blocks of all stripes, [stripe][shard][tail].  rsEncodeParityBlockedBatch /
     * rsDecodeMissingBlockedBatch run over device pools in that layout,
     * {@link EcxBlockedStripes} over direct host buffers in it.
     */
    public static long[] blockedLayout(int dataShards, int parityShards, long byteCount) {
        long[] layout = new long[3];
        check(EcxNative.rsBlockedLayout(dataShards, parityShards, byteCount, layout));
        return layout;
    }

    /** Creates the codec handle of ReedSolomon.create(k, m) (ReedSolomon.java:34-61). */
    public static long createReedSolomon(int dataShards, int parityShards) {
        long[] h = new long[1];
        check(EcxNative.rsCreate(dataShards, parityShards, h));
        return h[0];
    }
}
