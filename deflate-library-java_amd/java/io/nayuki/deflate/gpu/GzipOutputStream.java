/*
 * Drop-in for io.nayuki.deflate.GzipOutputStream (D/GzipOutputStream.java:19-80) over the GPU
 * DeflaterOutputStream: the same constructors (a plain OutputStream gets the default deflater, as
 * D/GzipOutputStream.java:32-34), header written by the reference's own GzipMetadata.write, CRC-32
 * and ISIZE (mod 2^32) trailer, little-endian.  The CRC is fused into the GPU encoder when the
 * deflater is fresh (ndfl_deflate_chunks crc_inout, one pass over the data in HBM); a deflater that
 * already holds data keeps java.util.zip.CRC32 over the bytes written here, as the reference does.
 */
package io.nayuki.deflate.gpu;

import java.io.IOException;
import java.io.OutputStream;
import java.util.Objects;
import java.util.zip.CRC32;
import io.nayuki.deflate.GzipMetadata;


public final class GzipOutputStream extends OutputStream {
	
	private DeflaterOutputStream output;
	private final CRC32 hostCrc;         // null: the encoder computes the CRC
	private long length = 0;             // ISIZE is this mod 2^32
	private boolean ended = false;
	
	
	public GzipOutputStream(OutputStream out, GzipMetadata meta) throws IOException {
		this(new DeflaterOutputStream(out), meta);
	}
	
	
	public GzipOutputStream(DeflaterOutputStream out, GzipMetadata meta) throws IOException {
		Objects.requireNonNull(out);
		Objects.requireNonNull(meta);
		meta.write(out.getUnderlyingStream());
		output = out;
		hostCrc = out.enableCrc() ? null : new CRC32();
	}
	
	
	@Override public void write(int b) throws IOException {
		write(new byte[]{(byte)b}, 0, 1);
	}
	
	
	@Override public void write(byte[] b, int off, int len) throws IOException {
		if (ended)
			throw new IllegalStateException("Stream already ended");
		output.write(b, off, len);
		if (hostCrc != null)
			hostCrc.update(b, off, len);
		length += len;
	}
	
	
	public void finish() throws IOException {
		if (ended)
			throw new IllegalStateException("Stream already ended");
		output.finish();
		ended = true;
		int crc = hostCrc != null ? (int)hostCrc.getValue() : output.crc();
		var trailer = new byte[8];
		for (int i = 0; i < 4; i++) {
			trailer[i] = (byte)(crc >>> (8 * i));
			trailer[4 + i] = (byte)(length >>> (8 * i));
		}
		output.getUnderlyingStream().write(trailer);
	}
	
	
	@Override public void close() throws IOException {
		if (output == null)
			return;
		if (!ended)
			finish();
		output.close();
		output = null;
	}
	
}
