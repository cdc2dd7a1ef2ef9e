/*
 * Drop-in for io.nayuki.deflate.ZlibOutputStream (D/ZlibOutputStream.java:18-77) over the GPU
 * DeflaterOutputStream: header by the reference's ZlibMetadata.write, Adler-32 trailer big-endian.
 * The checksum: ndfl_adler32 on the GPU for large arrays, a host loop for small ones.
 */
package io.nayuki.deflate.gpu;

import java.io.IOException;
import java.io.OutputStream;
import java.util.Objects;
import io.nayuki.deflate.ZlibMetadata;


public final class ZlibOutputStream extends OutputStream {
	
	private DeflaterOutputStream output;
	private NativeCodec codec;
	private int adler = 1;
	private boolean ended = false;
	
	
	public ZlibOutputStream(OutputStream out, ZlibMetadata meta) throws IOException {
		this(new DeflaterOutputStream(out), meta);
	}
	
	
	public ZlibOutputStream(DeflaterOutputStream out, ZlibMetadata meta) throws IOException {
		Objects.requireNonNull(out);
		Objects.requireNonNull(meta);
		meta.write(out.getUnderlyingStream());
		output = out;
	}
	
	
	@Override public void write(int b) throws IOException {
		write(new byte[]{(byte)b}, 0, 1);
	}
	
	
	@Override public void write(byte[] b, int off, int len) throws IOException {
		if (ended)
			throw new IllegalStateException("Stream already ended");
		output.write(b, off, len);
		if (len == 0)
			return;
		if (codec == null)
			codec = new NativeCodec(0);
		adler = codec.adler32(adler, b, off, len);
	}
	
	
	public void finish() throws IOException {
		if (ended)
			throw new IllegalStateException("Stream already ended");
		output.finish();
		ended = true;
		var trailer = new byte[4];
		for (int i = 0; i < 4; i++)
			trailer[i] = (byte)(adler >>> (24 - 8 * i));
		output.getUnderlyingStream().write(trailer);
	}
	
	
	@Override public void close() throws IOException {
		if (output == null)
			return;
		if (!ended)
			finish();
		output.close();
		output = null;
		if (codec != null)
			codec.close();
	}
	
}
