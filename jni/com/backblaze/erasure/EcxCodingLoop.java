package com.backblaze.erasure;

import com.backblaze.erasure.ecx.Ecx;
import com.backblaze.erasure.ecx.EcxNative;

/**
 * The reference's operator plug point (CodingLoop.java:79-117), executed by libecx.so
 * on the MI355X: {@code new ReedSolomon(k, m, new EcxCodingLoop())} (ReedSolomon.java:41)
 * runs encodeParity, decodeMissing and isParityCorrect through the GPU kernel with
 * the same results as InputOutputByteTableCodingLoop (every coefficient row arrives
 * with the call; the library caches the compiled plan per matrix content).
 */
public class EcxCodingLoop extends CodingLoopBase {

    @Override
    public void codeSomeShards(byte[][] matrixRows,
                               byte[][] inputs, int inputCount,
                               byte[][] outputs, int outputCount,
                               int offset, int byteCount) {
        byte[] rows = Ecx.flatten(matrixRows, outputCount, inputCount);
        Ecx.check(EcxNative.codeSomeShards(rows, inputs, null, inputCount, outputs, null, outputCount, offset,
                byteCount));
    }

    @Override
    public boolean checkSomeShards(byte[][] matrixRows,
                                   byte[][] inputs, int inputCount,
                                   byte[][] toCheck, int checkCount,
                                   int offset, int byteCount,
                                   byte[] tempBuffer) {
        byte[] rows = Ecx.flatten(matrixRows, checkCount, inputCount);
        return Ecx.check(EcxNative.checkSomeShards(rows, inputs, null, inputCount, toCheck, null, checkCount, offset,
                byteCount, tempBuffer)) == 1;
    }
}
