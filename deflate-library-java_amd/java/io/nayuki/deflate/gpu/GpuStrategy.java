/*
 * A Strategy (D/comp/Strategy.java:14) whose decisions are computed by libndfl.so: the library's
 * strategies as a tree -- Lz77Huffman and Uncompressed leaves encoded on the GPU, MultiStrategy and
 * BinarySplit composed exactly as D/comp/MultiStrategy.java:31-57 and D/comp/BinarySplit.java:30-82
 * do -- through ndfl_decide / ndfl_compress_to.  It plugs into the reference's own
 * DeflaterOutputStream(out, lookahead, history, strategy) chunk by chunk, and mixes with any other
 * Strategy inside the reference's MultiStrategy / BinarySplit.  (The batched stream path,
 * gpu.DeflaterOutputStream, is the fast one.)
 */
package io.nayuki.deflate.gpu;

import java.io.IOException;
import java.lang.ref.Cleaner;
import java.util.ArrayList;
import java.util.List;
import java.util.Objects;
import io.nayuki.deflate.comp.BitOutputStream;
import io.nayuki.deflate.comp.Decision;
import io.nayuki.deflate.comp.Lz77Huffman;
import io.nayuki.deflate.comp.Strategy;


public final class GpuStrategy implements Strategy {
	
	private static final Cleaner CLEANER = Cleaner.create();
	
	private final int[] nodes;      // ndfl_strategy_node x n (9 ints each), root at 0
	private final NativeCodec codec;
	
	
	private GpuStrategy(int[] nodes, NativeCodec codec) {
		this.nodes = nodes;
		this.codec = codec;
	}
	
	
	/*---- builders mirroring the reference's constructors ----*/
	
	public static GpuStrategy of(Lz77Huffman st, NativeCodec codec) {
		return new GpuStrategy(new int[]{NativeCodec.KIND_LZ77, st.useDynamicHuffmanCodes() ? 1 : 0,
			st.searchMinimumRunLength(), st.searchMaximumRunLength(), st.searchMinimumDistance(),
			st.searchMaximumDistance(), 0, 0, 0}, codec);
	}
	
	public static GpuStrategy uncompressed(NativeCodec codec) {
		return new GpuStrategy(new int[]{NativeCodec.KIND_UNCOMPRESSED, 0, 0, 0, 0, 0, 0, 0, 0}, codec);
	}
	
	public static GpuStrategy multi(GpuStrategy... strats) {
		Objects.requireNonNull(strats);
		if (strats.length == 0)
			throw new IllegalArgumentException("Empty list of strategies");
		// root, then the children's root nodes contiguously, then each child's remaining nodes
		List<int[]> out = new ArrayList<>();
		out.add(new int[]{NativeCodec.KIND_MULTI, 0, 0, 0, 0, 0, 1, strats.length, 0});
		int base = 1 + strats.length;
		int[][] rest = new int[strats.length][];
		for (int i = 0; i < strats.length; i++) {
			int[] sub = strats[i].relocated(base - 1);       // the child's node 0 sits at slot 1 + i
			out.add(java.util.Arrays.copyOfRange(sub, 0, 9));
			rest[i] = java.util.Arrays.copyOfRange(sub, 9, sub.length);
			base += rest[i].length / 9;
		}
		for (int[] r : rest)
			out.add(r);
		return new GpuStrategy(flatten(out), strats[0].codec);
	}
	
	public static GpuStrategy binarySplit(GpuStrategy strat, int minBlockLen) {
		Objects.requireNonNull(strat);
		if (minBlockLen < 1)
			throw new IllegalArgumentException("Non-positive minimum block length");
		List<int[]> out = new ArrayList<>();
		out.add(new int[]{NativeCodec.KIND_BINSPLIT, 0, 0, 0, 0, 0, 1, 0, minBlockLen});
		out.add(strat.relocated(1));
		return new GpuStrategy(flatten(out), strat.codec);
	}
	
	
	// this tree's nodes with child indices moved by `by` (node 0 goes to slot `by`)
	private int[] relocated(int by) {
		int[] r = nodes.clone();
		for (int i = 0; i < r.length; i += 9)
			if (r[i] == NativeCodec.KIND_MULTI || r[i] == NativeCodec.KIND_BINSPLIT)
				r[i + 6] += by;
		return r;
	}
	
	private static int[] flatten(List<int[]> parts) {
		int n = 0;
		for (int[] p : parts)
			n += p.length;
		int[] r = new int[n];
		int k = 0;
		for (int[] p : parts) {
			System.arraycopy(p, 0, r, k, p.length);
			k += p.length;
		}
		return r;
	}
	
	
	/*---- Strategy ----*/
	
	@Override public Decision decide(byte[] b, int off, int historyLen, int dataLen) {
		Objects.checkFromIndexSize(off, historyLen + dataLen, b.length);
		var bitLengths = new long[8];
		long dec = NativeCodec.decide0(codec.handle(), nodes, 0, b, off, historyLen, dataLen, bitLengths);
		var d = new GpuDecision(codec, dec, bitLengths);
		CLEANER.register(d, () -> NativeCodec.freeDecision0(dec));
		return d;
	}
	
	
	private static final class GpuDecision implements Decision {
		private final NativeCodec codec;
		private final long handle;
		private final long[] bitLengths;
		
		GpuDecision(NativeCodec codec, long handle, long[] bitLengths) {
			this.codec = codec;
			this.handle = handle;
			this.bitLengths = bitLengths;
		}
		
		@Override public long[] getBitLengths() {
			return bitLengths.clone();
		}
		
		@Override public void compressTo(BitOutputStream out, boolean isFinal) throws IOException {
			int p = out.getBitPosition();
			long max = 0;
			for (long x : bitLengths)
				max = Math.max(max, x);
			for (long cap = max / 8 + 4096; ; cap *= 2) {
				var buf = new byte[(int)Math.min(cap, Integer.MAX_VALUE - 8)];
				long end = NativeCodec.compressTo0(codec.handle(), handle, isFinal, p, buf);
				if (end < 0)
					continue;
				// bits [p, end) of buf, LSB first, in pieces of at most 24 bits
				for (long i = p; i < end; ) {
					int k = (int)Math.min(24, end - i);
					int v = 0;
					for (int j = 0; j < k; j++, i++)
						v |= ((buf[(int)(i >>> 3)] >>> (i & 7)) & 1) << j;
					out.writeBits(v, k);
				}
				return;
			}
		}
	}
	
}
