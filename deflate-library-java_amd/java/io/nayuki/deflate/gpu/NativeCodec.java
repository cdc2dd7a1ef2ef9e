/*
 * JNI facade over libndfl.so (include/ndfl.h); the glue is native/ndfl_jni.c.  One codec per stream
 * object, not thread-safe (the reference's streams are not either).  Built only where a JDK exists:
 * this image has none, so these sources are compiled by a maintainer, not by our tests.
 */
package io.nayuki.deflate.gpu;

import java.io.IOException;
import java.nio.ByteBuffer;


final class NativeCodec implements AutoCloseable {
	
	static {
		System.loadLibrary("ndfl");
		System.loadLibrary("ndfl_jni");
	}
	
	static final int NEED_INPUT = 64;        // NDFL_NEED_INPUT
	static final int E_CAPACITY = -3;        // NDFL_E_CAPACITY
	static final int E_UNSUPPORTED = -2;     // NDFL_E_UNSUPPORTED
	static final int KIND_LZ77 = 0, KIND_UNCOMPRESSED = 1, KIND_MULTI = 2, KIND_BINSPLIT = 3;
	
	private long ctx;
	
	
	NativeCodec(int device) throws IOException {
		ctx = create(device);
	}
	
	
	long handle() {
		if (ctx == 0)
			throw new IllegalStateException("Codec closed");
		return ctx;
	}
	
	
	@Override public void close() {
		if (ctx != 0) {
			destroy(ctx);
			ctx = 0;
		}
	}
	
	
	/*---- native entry points (ndfl_jni.c) ----*/
	
	static native long create(int device) throws IOException;
	static native void destroy(long ctx);
	
	// end bit in res[0]; returns 0 or a negative code not thrown (NDFL_E_CAPACITY / _UNSUPPORTED)
	static native int deflateChunks0(long ctx, ByteBuffer hist, int histLen, int histLimit, ByteBuffer data,
		long len, int chunkLen, int strategy, boolean isFinal, int startBitPos, ByteBuffer out, long[] res, int[] crc);
	static native int deflateChunksLz770(long ctx, ByteBuffer hist, int histLen, int histLimit, ByteBuffer data,
		long len, int chunkLen, boolean dynamic, int minRun, int maxRun, int minDist, int maxDist, boolean isFinal,
		int startBitPos, ByteBuffer out, long[] res, int[] crc);
	static native int deflateChunksMulti0(long ctx, ByteBuffer hist, int histLen, int histLimit, ByteBuffer data,
		long len, int chunkLen, int[] subs, boolean isFinal, int startBitPos, ByteBuffer out, long[] res, int[] crc);
	static native long deflateBound0(long len, int chunkLen);
	
	// res[0] = bytes decoded after the window, res[1] = consumed bits
	static native int inflateRange0(long ctx, ByteBuffer in, long inLen, long startBit, ByteBuffer out, long dictLen,
		boolean partial, long[] res);
	
	// the message of a decode's DataFormatException: ndfl_error_string(reason), with the reserved
	// symbol appended where the reference appends it, "Reserved run length symbol: " + sym /
	// "Reserved distance symbol: " + sym (D/decomp/Open.java:516, 550; ndfl_ctx_error_symbol)
	static native String errorMessage0(long ctx, int reason);
	
	static native int crc320(long ctx, int crc, ByteBuffer data, long len);
	static native int adler320(long ctx, int adler, ByteBuffer data, long len);
	
	
	static final int GPU_CHECKSUM_MIN = 1 << 20;   // smaller arrays: a host loop beats a launch + copy
	private ByteBuffer staging;
	
	// java.util.zip.Adler32.update continued from `adler` (the zlib streams' checksum,
	// D/ZlibOutputStream.java:48, D/ZlibInputStream.java:57): large arrays on the GPU (ndfl_adler32),
	// small ones on the host
	int adler32(int adler, byte[] b, int off, int len) {
		if (len >= GPU_CHECKSUM_MIN) {
			if (staging == null || staging.capacity() < len)
				staging = ByteBuffer.allocateDirect(len);
			staging.put(0, b, off, len);
			return adler320(handle(), adler, staging, len);
		}
		long s1 = adler & 0xFFFF, s2 = adler >>> 16;
		for (int i = 0; i < len; ) {
			int end = Math.min(len, i + 5552);       // no overflow before the reduction
			for (; i < end; i++) {
				s1 += b[off + i] & 0xFF;
				s2 += s1;
			}
			s1 %= 65521;
			s2 %= 65521;
		}
		return (int)((s2 << 16) | s1);
	}
	
	// the plugin API: strategy tree (9 ints per node) -> decision handle; compressTo -> end bit or -1
	static native long decide0(long ctx, int[] nodes, int root, byte[] b, int off, int historyLen, int dataLen,
		long[] bitLengths);
	static native long compressTo0(long ctx, long dec, boolean isFinal, int startBitPos, byte[] out);
	static native void freeDecision0(long dec);
	
}
