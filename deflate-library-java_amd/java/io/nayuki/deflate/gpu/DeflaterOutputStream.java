/*
 * Drop-in for io.nayuki.deflate.DeflaterOutputStream (D/DeflaterOutputStream.java:30-173) on the GPU:
 * same constructors, write / finish / close contract and exceptions, same bytes.  Writes are staged
 * in a direct buffer; when it holds more than BATCH bytes, all full chunks but the last go to ONE
 * ndfl_deflate_chunks* call (exact: each chunk's block depends only on raw input, SURVEY App. A.1);
 * the BitOut position and pending byte carry across calls as the reference's BitOut does
 * (:141-171).  Strategies the batched calls do not take run chunk by chunk through
 * Strategy.decide / Decision.compressTo exactly as the reference's writeBuffer (:119-137).
 */
package io.nayuki.deflate.gpu;

import java.io.IOException;
import java.io.OutputStream;
import java.nio.ByteBuffer;
import java.util.Objects;
import io.nayuki.deflate.comp.BitOutputStream;
import io.nayuki.deflate.comp.Lz77Huffman;
import io.nayuki.deflate.comp.Strategy;
import io.nayuki.deflate.comp.Uncompressed;


public final class DeflaterOutputStream extends OutputStream {
	
	static final int BATCH = 64 << 20;
	
	private OutputStream output;
	private final int dataLookaheadLimit, historyLookbehindLimit;
	private final Strategy strategy;
	private NativeCodec codec;           // created on first use (the constructors do no I/O)
	private ByteBuffer pending;          // staged data (direct)
	private final ByteBuffer history;    // last <= historyLookbehindLimit raw bytes (direct)
	private ByteBuffer outBuf;           // compressed staging (direct)
	private int bitPos = 0;              // BitOut bits pending (0..7)
	private int bitByte = 0;             // the pending partial byte
	private int[] crc = null;            // GzipOutputStream asks for the CRC pass fused into the encoder
	private long written = 0;            // bytes written so far
	private boolean ended = false;
	
	
	public DeflaterOutputStream(OutputStream out) {
		this(out, 64 * 1024, 32 * 1024, Lz77Huffman.RLE_DYNAMIC);
	}
	
	
	public DeflaterOutputStream(OutputStream out, int dataLookaheadLimit, int historyLookbehindLimit,
			Strategy strat) {
		output = Objects.requireNonNull(out);
		strategy = Objects.requireNonNull(strat);
		if (dataLookaheadLimit < 1 || historyLookbehindLimit < 0 || historyLookbehindLimit > 32 * 1024
				|| (long)dataLookaheadLimit + historyLookbehindLimit > Integer.MAX_VALUE)
			throw new IllegalArgumentException("Invalid capacities");
		this.dataLookaheadLimit = dataLookaheadLimit;
		this.historyLookbehindLimit = historyLookbehindLimit;
		pending = ByteBuffer.allocateDirect(Math.max(BATCH, dataLookaheadLimit) + dataLookaheadLimit + 1);
		history = ByteBuffer.allocateDirect(Math.max(historyLookbehindLimit, 1));
		history.limit(0);
	}
	
	
	// D/DeflaterOutputStream.java:69-73 (package-private there too; the gpu Gzip/Zlib streams use it)
	OutputStream getUnderlyingStream() {
		if (output == null)
			throw new IllegalStateException("Stream already closed");
		return output;
	}
	
	
	private NativeCodec codec() throws IOException {
		if (codec == null)
			codec = new NativeCodec(0);
		return codec;
	}
	
	
	// GzipOutputStream: fuse the CRC-32 of the data into the encoder (ndfl_deflate_chunks crc_inout).
	// Only before the first write, so the CRC covers exactly the bytes written through the gzip stream;
	// returns false otherwise (the caller keeps its own java.util.zip.CRC32).
	boolean enableCrc() {
		if (written != 0 || crc != null)
			return false;
		crc = new int[]{0};
		return true;
	}
	
	
	// the CRC-32 of everything written; valid after finish()
	int crc() {
		return crc[0];
	}
	
	
	@Override public void write(int b) throws IOException {
		write(new byte[]{(byte)b}, 0, 1);
	}
	
	
	@Override public void write(byte[] b, int off, int len) throws IOException {
		if (ended)
			throw new IllegalStateException("Stream already ended");
		Objects.checkFromIndexSize(off, len, b.length);
		written += len;
		while (len > 0) {
			if (!pending.hasRemaining())
				flush(false);
			int n = Math.min(len, pending.remaining());
			pending.put(b, off, n);
			off += n;
			len -= n;
		}
		if (pending.position() > BATCH)
			flush(false);
	}
	
	
	public void finish() throws IOException {
		if (ended)
			throw new IllegalStateException("Stream already ended");
		flush(true);
		if (bitPos > 0)
			output.write(bitByte);                  // BitOut.finish zero-pads (:164-169)
		bitPos = 0;
		ended = true;
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
	
	
	// compress the staged chunks: all full chunks except the last when !isFinal (the reference
	// flushes a chunk only once more data arrives), everything when isFinal
	private void flush(boolean isFinal) throws IOException {
		int n = pending.position();
		int take = isFinal ? n : (n - 1) / dataLookaheadLimit * dataLookaheadLimit;
		if (!isFinal && take == 0)
			return;
		ByteBuffer data = pending.duplicate();
		data.flip().limit(take);
		long bound = NativeCodec.deflateBound0(take, dataLookaheadLimit) + 16;
		if (outBuf == null || outBuf.capacity() < bound)
			outBuf = ByteBuffer.allocateDirect((int)Math.min(bound, Integer.MAX_VALUE - 8));
		var res = new long[1];
		int r = batched(data.slice(), take, isFinal, res);
		if (r == NativeCodec.E_UNSUPPORTED) {
			perChunk(data.slice(), take, isFinal);
		} else {
			long endBits = res[0];
			int whole = (int)(endBits >>> 3);
			byte[] bytes = new byte[(int)((endBits + 7) >>> 3)];
			outBuf.get(0, bytes);
			if (bytes.length > 0)
				bytes[0] |= (byte)bitByte;
			output.write(bytes, 0, whole);
			bitPos = (int)(endBits & 7);
			bitByte = bitPos > 0 ? bytes[whole] & 0xFF : 0;
		}
		// history: the last min(limit, pos) raw bytes
		updateHistory(data, take);
		pending.flip().position(take);
		pending.compact();
	}
	
	
	private int batched(ByteBuffer data, int take, boolean isFinal, long[] res) throws IOException {
		int histLen = history.limit();
		long ctx = codec().handle();
		if (strategy instanceof Lz77Huffman lz) {
			return NativeCodec.deflateChunksLz770(ctx, history, histLen, historyLookbehindLimit, data, take,
				dataLookaheadLimit, lz.useDynamicHuffmanCodes(), lz.searchMinimumRunLength(), lz.searchMaximumRunLength(),
				lz.searchMinimumDistance(), lz.searchMaximumDistance(), isFinal, bitPos, outBuf, res, crc);
		} else if (strategy == Uncompressed.SINGLETON) {
			return NativeCodec.deflateChunks0(ctx, history, histLen, historyLookbehindLimit, data, take,
				dataLookaheadLimit, 6 /* NDFL_UNCOMPRESSED */, isFinal, bitPos, outBuf, res, crc);
		}
		return NativeCodec.E_UNSUPPORTED;        // any other Strategy: chunk by chunk
	}
	
	
	// DeflaterOutputStream.writeBuffer (:119-137) per chunk, over the staged bytes
	private void perChunk(ByteBuffer data, int take, boolean isFinal) throws IOException {
		var bo = new BitOut();
		int hl = history.limit();
		var combined = new byte[hl + Math.max(dataLookaheadLimit, 1)];
		history.get(0, combined, 0, hl);
		int pos = 0;
		do {
			int k = Math.min(dataLookaheadLimit, take - pos);
			data.get(pos, combined, hl, k);
			strategy.decide(combined, 0, hl, k).compressTo(bo, isFinal && pos + k == take);
			if (crc != null)
				crc[0] = NativeCodec.crc320(codec().handle(), crc[0], ByteBuffer.allocateDirect(k).put(0, combined, hl, k), k);
			int nh = Math.min(historyLookbehindLimit, hl + k);
			System.arraycopy(combined, hl + k - nh, combined, 0, nh);
			hl = nh;
			pos += k;
		} while (pos < take);
	}
	
	
	private void updateHistory(ByteBuffer data, int take) {
		if (historyLookbehindLimit == 0)
			return;
		int keepOld = Math.max(0, Math.min(history.limit(), historyLookbehindLimit - take));
		var tmp = new byte[keepOld + Math.min(take, historyLookbehindLimit)];
		history.get(history.limit() - keepOld, tmp, 0, keepOld);
		data.get(take - (tmp.length - keepOld), tmp, keepOld, tmp.length - keepOld);
		history.clear();
		history.put(tmp).flip();
	}
	
	
	// BitOut (D/DeflaterOutputStream.java:141-171) for the per-chunk path, continuing the stream's
	// pending bits
	private final class BitOut implements BitOutputStream {
		@Override public void writeBits(int value, int numBits) throws IOException {
			for (int i = 0; i < numBits; i++) {
				bitByte |= ((value >>> i) & 1) << bitPos;
				if (++bitPos == 8) {
					output.write(bitByte);
					bitByte = 0;
					bitPos = 0;
				}
			}
		}
		
		@Override public int getBitPosition() {
			return bitPos;
		}
	}
	
}
