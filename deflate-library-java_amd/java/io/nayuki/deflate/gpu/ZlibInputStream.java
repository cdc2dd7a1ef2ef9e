/*
 * Drop-in for io.nayuki.deflate.ZlibInputStream (D/ZlibInputStream.java:21-99) over the GPU
 * InflaterInputStream: header by the reference's ZlibMetadata.read, DEFLATE data with endExactly,
 * big-endian Adler-32 trailer checked with the reference's Reason and message.  The checksum:
 * ndfl_adler32 on the GPU for large reads, a host loop for small ones.
 */
package io.nayuki.deflate.gpu;

import java.io.BufferedInputStream;
import java.io.IOException;
import java.io.InputStream;
import java.util.Objects;
import io.nayuki.deflate.DataFormatException;
import io.nayuki.deflate.DataFormatException.Reason;
import io.nayuki.deflate.ZlibMetadata;


public final class ZlibInputStream extends InputStream {
	
	private InputStream rawInput;
	private InflaterInputStream inflater;        // null once the DEFLATE data has ended
	private final ZlibMetadata metadata;
	private NativeCodec codec;
	private int adler = 1;
	
	
	public ZlibInputStream(InputStream in) throws IOException {
		Objects.requireNonNull(in);
		metadata = ZlibMetadata.read(in);
		rawInput = in.markSupported() ? in : new BufferedInputStream(in);
		inflater = new InflaterInputStream(rawInput, true);
	}
	
	
	public ZlibMetadata getMetadata() {
		return metadata;
	}
	
	
	@Override public int read() throws IOException {
		var b = new byte[1];
		int n = read(b, 0, 1);
		return n == 1 ? b[0] & 0xFF : -1;
	}
	
	
	@Override public int read(byte[] b, int off, int len) throws IOException {
		if (inflater == null)
			return -1;
		int n = inflater.read(b, off, len);
		if (n > 0) {
			if (codec == null)
				codec = new NativeCodec(0);
			adler = codec.adler32(adler, b, off, n);
		}
		if (n != -1)
			return n;
		inflater = null;
		var t = new byte[4];
		if (rawInput.readNBytes(t, 0, 4) != 4)
			throw DataFormatException.throwUnexpectedEnd();
		int expect = ((t[0] & 0xFF) << 24) | ((t[1] & 0xFF) << 16) | ((t[2] & 0xFF) << 8) | (t[3] & 0xFF);
		if (adler != expect)
			throw new DataFormatException(Reason.DECOMPRESSED_CHECKSUM_MISMATCH, "Decompression Adler-32 mismatch");
		return -1;
	}
	
	
	@Override public void close() throws IOException {
		if (rawInput != null)
			rawInput.close();
		rawInput = null;
		inflater = null;
		if (codec != null)
			codec.close();
	}
	
}
