package distributed.erasure.coding.clay;

import com.backblaze.erasure.ecx.Ecx;
import com.backblaze.erasure.ecx.EcxNative;

import java.nio.ByteBuffer;

/**
 * ClayCodeErasureDecodingStep (ClayCodeErasureDecodingStep.java:28-107) on libecx.so:
 * the same constructor arguments (erased indexes, and the code's k and m instead of
 * the two ReedSolomon objects, which the library builds identically), the same
 * performCoding(ECChunk[], ECChunk[]) contract (inputs n*alpha plane-major, null =
 * erased or absent; outputs |E|*alpha), and a batched form over many stripes for the
 * coordinator (ClayCoordinator.kt:96-97) -- device-resident or in (direct) host memory.
 * Results are those of the reference's decode/encode stage sequence; deviations
 * affect only caller-visible side effects (DESIGN.md section 5).
 */
public class EcxClayCodeErasureDecodingStep {
    private long clay;  // 0 once closed
    private final int numErased;

    public EcxClayCodeErasureDecodingStep(int[] erasedIndexes, int numDataUnits, int numParityUnits) {
        long[] h = new long[1];
        Ecx.check(EcxNative.clayCreate(numDataUnits, numParityUnits, erasedIndexes, erasedIndexes.length, h));
        this.clay = h[0];
        this.numErased = erasedIndexes.length;
    }

    /** Sub-packetization alpha (ClayCodeUtil, ClayCodeErasureDecodingStep.java:690-695). */
    public int subPacketSize() {
        int[] q = new int[1], t = new int[1], alpha = new int[1];
        Ecx.check(EcxNative.clayGeometry(handle(), q, t, alpha));
        return alpha[0];
    }

    /**
     * performCoding(ECChunk[], ECChunk[]) (ClayCodeErasureDecodingStep.java:53-107).  Heap
     * buffers are passed by array and position; as the reference, input positions
     * advance by the buffer size and output positions are left where they were.
     */
    public void performCoding(ECChunk[] inputChunks, ECChunk[] outputChunks) {
        ByteBuffer[] in = ECChunk.toBuffers(inputChunks);
        ByteBuffer[] out = ECChunk.toBuffers(outputChunks);
        int bufSize = -1;
        for (ByteBuffer b : in) {
            if (b != null) {
                bufSize = b.remaining();
                break;
            }
        }
        if (bufSize < 0) {
            throw new IllegalArgumentException("Invalid buffer, all null");
        }
        byte[][] inArrays = new byte[in.length][];
        int[] inPos = new int[in.length];
        for (int i = 0; i < in.length; i++) {
            if (in[i] != null) {
                inArrays[i] = in[i].array();
                inPos[i] = in[i].arrayOffset() + in[i].position();
            }
        }
        byte[][] outArrays = new byte[out.length][];
        int[] outPos = new int[out.length];
        for (int i = 0; i < out.length; i++) {
            outArrays[i] = out[i].array();
            outPos[i] = out[i].arrayOffset() + out[i].position();
        }
        Ecx.check(EcxNative.clayPerformCoding(handle(), inArrays, inPos, outArrays, outPos, bufSize));
        for (ByteBuffer b : in) {
            if (b != null) {
                b.position(b.position() + bufSize);
            }
        }
    }

    /**
     * Batched performCoding over {@code nstripes} device-resident stripes (HBM addresses):
     * stripe s's sub-chunk slot z*n+node at in + s*inStripeStride + slot*inSubStride, its
     * repaired sub-chunk z*|E|+j at out + s*outStripeStride + slot*outSubStride.  Enqueued on
     * {@code stream} (a hipStream_t, 0 = the default stream).
     */
    public void performCodingBatch(long in, long inStripeStride, long inSubStride, long out, long outStripeStride,
                                   long outSubStride, long nstripes, long bufSize, long stream) {
        Ecx.check(EcxNative.clayPerformCodingBatch(handle(), in, inStripeStride, inSubStride, out, outStripeStride,
                outSubStride, nstripes, bufSize, stream));
    }

    /**
     * The same from direct host ByteBuffers (pipelined over PCIe; synchronous), addressed
     * from each buffer's start.  Each buffer must hold (nstripes-1)*stripeStride +
     * maxSlot*subStride + bufSize bytes, maxSlot being the highest sub-chunk slot the
     * repair reads (inputs) or writes (outputs): a shorter buffer throws
     * ArrayIndexOutOfBoundsException before anything is read, as the reference's
     * ByteBuffer get/put would (ClayCoordinator.kt:378-390); a heap (non-direct) buffer
     * throws NullPointerException.  The check is repeated natively from the buffers'
     * capacities (EcxNative.clayPerformCodingBatchHostBuffer).
     */
    public void performCodingBatchHost(ByteBuffer in, long inStripeStride, long inSubStride, ByteBuffer out,
                                       long outStripeStride, long outSubStride, long nstripes, long bufSize) {
        if (nstripes < 0 || bufSize < 0 || inStripeStride < 0 || inSubStride < 0 || outStripeStride < 0
                || outSubStride < 0) {
            throw new IllegalArgumentException("negative batch count, size or stride");
        }
        if (numErased > 0 && nstripes > 0 && bufSize > 0) {
            int[] slots = maxSlots();
            checkExtent(in, "input", inStripeStride, inSubStride, slots[0], nstripes, bufSize);
            checkExtent(out, "output", outStripeStride, outSubStride, slots[1], nstripes, bufSize);
        }
        Ecx.check(EcxNative.clayPerformCodingBatchHostBuffer(handle(), in, inStripeStride, inSubStride, out,
                outStripeStride, outSubStride, nstripes, bufSize));
    }

    /**
     * performCodingBatchHost split over several GPUs of this process (SURVEY.md 8(e)): device
     * j of {@code devices} repairs the contiguous stripe range j of devices.length (the
     * remainder on the first ranges) with a host thread, streams and buffer ring of its own;
     * returns when every device has finished.  Same buffer contract and checks as
     * performCodingBatchHost; an unknown device id throws IllegalArgumentException before
     * anything is copied.
     */
    public void performCodingBatchHostDevices(ByteBuffer in, long inStripeStride, long inSubStride, ByteBuffer out,
                                              long outStripeStride, long outSubStride, long nstripes, long bufSize,
                                              int[] devices) {
        if (devices == null || devices.length == 0) {
            throw new IllegalArgumentException("no devices");
        }
        if (nstripes < 0 || bufSize < 0 || inStripeStride < 0 || inSubStride < 0 || outStripeStride < 0
                || outSubStride < 0) {
            throw new IllegalArgumentException("negative batch count, size or stride");
        }
        if (numErased > 0 && nstripes > 0 && bufSize > 0) {
            int[] slots = maxSlots();
            checkExtent(in, "input", inStripeStride, inSubStride, slots[0], nstripes, bufSize);
            checkExtent(out, "output", outStripeStride, outSubStride, slots[1], nstripes, bufSize);
        }
        Ecx.check(EcxNative.clayPerformCodingBatchHostDevicesBuffer(handle(), in, inStripeStride, inSubStride, out,
                outStripeStride, outSubStride, nstripes, bufSize, devices, devices.length));
    }

    /** Highest input and output sub-chunk slot of the repair (ecx_map_slot_extent). */
    private int[] maxSlots() {
        long[] m = new long[1];
        Ecx.check(EcxNative.clayMap(handle(), m));
        int[] in = new int[1], out = new int[1];
        Ecx.check(EcxNative.mapSlotExtent(m[0], in, out));
        return new int[] {in[0], out[0]};
    }

    private static void checkExtent(ByteBuffer b, String what, long stripeStride, long subStride, int maxSlot,
                                    long nstripes, long bufSize) {
        if (b == null || !b.isDirect()) {
            throw new NullPointerException(what + ": a direct ByteBuffer is required");
        }
        if (maxSlot < 0) {
            return;
        }
        long need;
        try {
            need = Math.addExact(Math.addExact(Math.multiplyExact(nstripes - 1, stripeStride),
                    Math.multiplyExact((long) maxSlot, subStride)), bufSize);
        } catch (ArithmeticException e) {
            throw new ArrayIndexOutOfBoundsException(what + ": batch extent overflows");
        }
        if (need > b.capacity()) {
            throw new ArrayIndexOutOfBoundsException(what + ": the batch addresses " + need
                    + " bytes but the buffer holds " + b.capacity());
        }
    }

    public int numErased() {
        return numErased;
    }

    private long handle() {
        if (clay == 0) {
            throw new IllegalStateException("EcxClayCodeErasureDecodingStep is closed");
        }
        return clay;
    }

    /**
     * Releases this step's reference to the native decoding step.  Idempotent: equal steps
     * share one reference-counted native object (ecx_clay_create), so a second release would
     * drop another step's reference; later calls on this step throw IllegalStateException.
     */
    public synchronized void close() {
        if (clay == 0) {
            return;
        }
        long h = clay;
        clay = 0;
        EcxNative.clayDestroy(h);
    }
}
