/*
 * Drop-in for io.nayuki.deflate.InflaterInputStream (D/InflaterInputStream.java:26-181) on the GPU.
 * The underlying stream is read in batches of at least inBufLen (default 64 MiB) bytes; each batch
 * is decoded by ndfl_inflate_range with NDFL_IN_PARTIAL, which stops at the last block boundary the
 * batch completes -- Open.read's incremental refill (D/decomp/Open.java:137-192) at block
 * granularity -- and the decode continues from that bit with the last 32 KiB of output as the
 * window (the reference's dictionary ring, :592-603).  With endExactly the underlying stream is
 * reset to its mark and skipped to the byte after the final block (Open.finish, :113-124).
 * Errors: a Reason code raises DataFormatException from the read call that reaches it, as Open.read
 * throws from inside the call (D/decomp/Open.java:83-110): a read asking for more bytes than remain
 * before the error copies them into b uncounted and throws; a read ending at or before the error
 * returns normally.  DataFormatException is unchecked (D/DataFormatException.java:15), so it is not
 * sticky; an IOException of the underlying stream is (:152-159).
 * Memory: with endExactly the underlying stream's mark is moved along with the consumed input
 * (reset, skip the consumed bytes, mark again, skip back to the read position), so a
 * BufferedInputStream holds at most about one batch, whatever the member's length -- the reference
 * marks again on every fill (D/decomp/Open.java:184).
 */
package io.nayuki.deflate.gpu;

import java.io.IOException;
import java.io.InputStream;
import java.nio.ByteBuffer;
import java.util.Objects;
import io.nayuki.deflate.DataFormatException;


public final class InflaterInputStream extends InputStream {
	
	static final int BATCH = 64 << 20;
	private static final int WINDOW = 32768;
	private static final long MAX_OUT = Integer.MAX_VALUE - 8;   // largest direct buffer
	
	private InputStream input;
	private final boolean endExactly;
	private final int batch;
	private NativeCodec codec;           // created on first use (the constructors do no I/O)
	private ByteBuffer in;               // unconsumed input (direct); byte 0 holds bit `bit` of the stream
	private int bit = 0;
	private boolean eof = false, last = false;
	private ByteBuffer out;              // window ++ decoded batch (direct)
	private int outPos = 0, outEnd = 0, windowLen = 0;
	private DataFormatException error = null;
	private IOException sticky = null;
	private boolean closed = false;
	
	
	public InflaterInputStream(InputStream in) {
		this(in, false);
	}
	
	
	public InflaterInputStream(InputStream in, boolean endExactly) {
		this(in, endExactly, 16 * 1024);
	}
	
	
	public InflaterInputStream(InputStream in, boolean endExactly, int inBufLen) {
		input = Objects.requireNonNull(in);
		if (inBufLen <= 0)
			throw new IllegalArgumentException("Non-positive input buffer size");
		batch = Math.max(inBufLen, BATCH);
		if (endExactly) {
			if (!in.markSupported())
				throw new IllegalArgumentException("Input stream not markable, cannot support detachment");
			markLimit = batch + MARK_SLACK;
			in.mark(markLimit);
		}
		this.endExactly = endExactly;
		this.in = ByteBuffer.allocateDirect(batch + 256);
		this.in.limit(0);
	}
	
	
	@Override public int read() throws IOException {
		var b = new byte[1];
		return switch (read(b)) {
			case  1 -> b[0] & 0xFF;
			case -1 -> -1;
			default -> throw new AssertionError("Unreachable value");
		};
	}
	
	
	@Override public int read(byte[] b, int off, int len) throws IOException {
		Objects.requireNonNull(b);
		Objects.checkFromIndexSize(off, len, b.length);
		if (closed)
			throw new IllegalStateException("Stream already closed");
		if (sticky != null)
			throw sticky;
		int result = 0;
		while (result < len) {
			if (outPos == outEnd) {
				if (error != null || last)
					break;
				try {
					fill();
				} catch (IOException e) {
					sticky = e;
					throw e;
				}
				continue;
			}
			int n = Math.min(len - result, outEnd - outPos);
			out.get(outPos, b, off + result, n);
			outPos += n;
			result += n;
		}
		if (result < len && error != null)
			throw error;                    // the bytes before the error are in b, uncounted
		if (result == 0 && len > 0)
			return -1;
		return (result > 0 || !last || outPos < outEnd) ? result : -1;
	}
	
	
	// decode the next batch (D/decomp/Open.java:83-124 over a bounded input buffer)
	private void fill() throws IOException {
		// the previous batch is fully served: its last <= 32 KiB become the window
		if (outEnd > 0) {
			int keep = Math.min(WINDOW, outEnd);
			var w = new byte[keep];
			out.get(outEnd - keep, w);
			out.put(0, w);
			windowLen = keep;
			outPos = outEnd = 0;
		}
		if (codec == null)
			codec = new NativeCodec(0);
		int want = batch;
		while (true) {
			readMore(want);
			final long all = in.limit();
			long inLen = all, over = all;
			var res = new long[2];
			int r;
			while (true) {
				// decode a prefix of the buffered input: all of it, unless its output would not fit in
				// one direct buffer -- then a shorter prefix, which stops at an earlier block boundary
				long need = windowLen + 4 * inLen + 65536;
				boolean partial = !eof || inLen < all;
				while (true) {
					prepareOut(Math.min(need, MAX_OUT));
					r = NativeCodec.inflateRange0(codec.handle(), in, inLen, bit, out, windowLen, partial, res);
					if (r != NativeCodec.E_CAPACITY || windowLen + res[0] + 16 > MAX_OUT)
						break;
					need = windowLen + res[0] + 16;
				}
				if (r != NativeCodec.E_CAPACITY)
					break;
				if (inLen <= 1)
					throw new IOException("A single DEFLATE block decodes to more than " + MAX_OUT + " bytes");
				over = inLen;                       // the shortest prefix known to overflow
				inLen /= 2;
			}
			if (r == NativeCodec.NEED_INPUT && res[0] == 0 && res[1] == bit && inLen < all) {
				// the shorter prefix completes no block, a longer one overflowed: search between them
				// for a prefix that completes a block within MAX_OUT; there is none only when the
				// first block alone decodes to more than MAX_OUT
				long lo = inLen, hi = over;
				boolean found = false;
				while (hi - lo > 1 && !found) {
					long mid = lo + (hi - lo) / 2;
					prepareOut(Math.min(windowLen + 4 * mid + 65536, MAX_OUT));
					r = NativeCodec.inflateRange0(codec.handle(), in, mid, bit, out, windowLen, true, res);
					if (r == NativeCodec.E_CAPACITY && windowLen + res[0] + 16 <= MAX_OUT) {
						prepareOut(windowLen + res[0] + 16);
						r = NativeCodec.inflateRange0(codec.handle(), in, mid, bit, out, windowLen, true, res);
					}
					if (r == NativeCodec.E_CAPACITY)
						hi = mid;
					else if (r == NativeCodec.NEED_INPUT && res[0] == 0 && res[1] == bit)
						lo = mid;
					else
						found = true;
				}
				if (!found)
					throw new IOException("A single DEFLATE block decodes to more than " + MAX_OUT + " bytes");
			}
			if (r == NativeCodec.NEED_INPUT && res[0] == 0 && res[1] == bit) {
				// no block completed: read more.  The next attempt re-decodes the incomplete block from
				// its start, so it waits for at least as much new input again (or for the source to
				// run dry, see readMore)
				final long cap = Integer.MAX_VALUE - 512L - MARK_SLACK;
				if (in.limit() >= cap)   // the buffer cannot grow: without this, fill() would retry forever
					throw new IOException("A single DEFLATE block needs more than " + cap + " bytes of input");
				want = (int)Math.min(cap, in.limit() + Math.max((long)batch, in.limit()));
				continue;
			}
			outPos = windowLen;
			outEnd = windowLen + (int)res[0];
			long bits = res[1];
			if (r == NativeCodec.NEED_INPUT) {
				consume((int)(bits >>> 3));
				bit = (int)(bits & 7);
			} else if (r == 0) {
				last = true;
				if (endExactly) {
					// Open.finish: reset to the mark, skip the bytes consumed (a partly used byte counts)
					int used = (int)((bits + 7) >>> 3);
					input.reset();
					input.skipNBytes(consumedBefore + used - markPos);
				}
			} else {
				error = new DataFormatException(DataFormatException.Reason.values()[r - 1],
					NativeCodec.errorMessage0(codec.handle(), r));
			}
			return;
		}
	}
	
	
	private long consumedBefore = 0;     // input bytes dropped from the front of `in`
	
	private static final int MARK_SLACK = 1 << 16;
	private long markPos = 0;            // stream position of the underlying stream's mark (endExactly)
	private int markLimit = 0;
	
	private void readMore(int want) throws IOException {
		if (in.capacity() < want + 256) {
			var bigger = ByteBuffer.allocateDirect(want + 256);
			bigger.put(in.duplicate().position(0).limit(in.limit())).flip();
			in = bigger;
		}
		if (endExactly && (consumedBefore != markPos || want + MARK_SLACK > markLimit)) {
			// move the mark to the first unconsumed byte: the bytes after it are all a reset may
			// need, and a BufferedInputStream keeps no more than that (served from its buffer)
			input.reset();
			input.skipNBytes(consumedBefore - markPos);
			markLimit = Math.max(want, batch) + MARK_SLACK;
			input.mark(markLimit);
			input.skipNBytes(in.limit());
			markPos = consumedBefore;
		}
		// read until `want` bytes are buffered or the stream ends.  A short read ends the read-ahead
		// early only when nothing more is ready (available() == 0: a pipe or socket whose peer may be
		// waiting for our output): what is buffered is decoded first, as Open decodes from whatever
		// its fill returned (D/decomp/Open.java:181-192); with data waiting the read-ahead goes on to
		// the batch, so a fast producer gets one GPU decode per batch, not one per pipe read
		var tmp = new byte[65536];
		while (in.limit() < want && !eof) {
			int ask = Math.min(tmp.length, want - in.limit());
			int n = input.read(tmp, 0, ask);
			if (n == -1)
				eof = true;
			else {
				int p = in.limit();
				in.limit(p + n);
				in.put(p, tmp, 0, n);
				if (n < ask && in.limit() > 0 && input.available() == 0)
					break;
			}
		}
	}
	
	private void consume(int bytes) {
		var rest = in.duplicate().position(bytes).limit(in.limit()).slice();
		int n = rest.remaining();
		var tmp = new byte[n];
		rest.get(tmp);
		in.clear();
		in.put(tmp).flip();
		consumedBefore += bytes;
	}
	
	private void prepareOut(long need) {
		if (out == null || out.capacity() < need) {
			var bigger = ByteBuffer.allocateDirect((int)Math.min(need, Integer.MAX_VALUE - 8));
			if (out != null && windowLen > 0) {
				var w = new byte[windowLen];
				out.get(0, w);
				bigger.put(0, w);
			}
			out = bigger;
		}
	}
	
	
	@Override public void close() throws IOException {
		if (!closed)
			input.close();
		closed = true;
		if (codec != null)
			codec.close();
	}
	
}
