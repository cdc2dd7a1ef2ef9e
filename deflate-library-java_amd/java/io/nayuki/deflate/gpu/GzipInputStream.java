/*
 * Drop-in for io.nayuki.deflate.GzipInputStream (D/GzipInputStream.java:22-100) over the GPU
 * InflaterInputStream: header parsed by the reference's GzipMetadata.read, the member's DEFLATE
 * data decoded with endExactly (the underlying stream is wrapped in a BufferedInputStream when it
 * cannot mark, as D/GzipInputStream.java:41-43), then the little-endian CRC-32 / ISIZE trailer
 * checked with the reference's Reasons and messages.  One member only; trailing bytes are left
 * unread, as in the reference.
 */
package io.nayuki.deflate.gpu;

import java.io.BufferedInputStream;
import java.io.IOException;
import java.io.InputStream;
import java.util.Objects;
import java.util.zip.CRC32;
import io.nayuki.deflate.DataFormatException;
import io.nayuki.deflate.DataFormatException.Reason;
import io.nayuki.deflate.GzipMetadata;


public final class GzipInputStream extends InputStream {
	
	private InputStream rawInput;
	private InflaterInputStream inflater;        // null once the DEFLATE data has ended
	private final GzipMetadata metadata;
	private CRC32 crc = new CRC32();
	private long length = 0;
	
	
	public GzipInputStream(InputStream in) throws IOException {
		Objects.requireNonNull(in);
		metadata = GzipMetadata.read(in);
		rawInput = in.markSupported() ? in : new BufferedInputStream(in);
		inflater = new InflaterInputStream(rawInput, true);
	}
	
	
	public GzipMetadata getMetadata() {
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
		if (n != -1) {
			crc.update(b, off, n);
			length += n;
			return n;
		}
		inflater = null;
		var t = new byte[8];
		if (rawInput.readNBytes(t, 0, 8) != 8)
			throw DataFormatException.throwUnexpectedEnd();
		int expectCrc = 0, expectLen = 0;
		for (int i = 3; i >= 0; i--) {
			expectCrc = (expectCrc << 8) | (t[i] & 0xFF);
			expectLen = (expectLen << 8) | (t[4 + i] & 0xFF);
		}
		if ((int)crc.getValue() != expectCrc)
			throw new DataFormatException(Reason.DECOMPRESSED_CHECKSUM_MISMATCH, "Decompression CRC-32 mismatch");
		if ((int)length != expectLen)
			throw new DataFormatException(Reason.DECOMPRESSED_SIZE_MISMATCH, "Decompressed size mismatch");
		return -1;
	}
	
	
	@Override public void close() throws IOException {
		if (rawInput != null)
			rawInput.close();
		rawInput = null;
		inflater = null;
	}
	
}
