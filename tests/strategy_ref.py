"""Test-side restatement of the reference's compressor plugin API (checker only): Decision trees of
D/comp/Uncompressed.java:22-51, D/comp/MultiStrategy.java:31-57 and D/comp/BinarySplit.java:36-82
over Lz77Huffman-preset leaves whose blocks come from the C oracle (oracle/ndfl_oracle.c restates
D/comp/Lz77Huffman.java), and DeflaterOutputStream's chunk loop (D/DeflaterOutputStream.java:76-137)
with its BitOut (:141-171).  Composes the same streams as ndfl.plugin / ndfl_decide, written
independently of them."""
import oracle_lib as O

LONG_MAX = (1 << 63) - 1


class BitWriter:
    def __init__(self):
        self.v = 0
        self.n = 0

    def writeBits(self, value, numBits):
        assert 0 <= numBits <= 31 and value >> numBits == 0
        self.v |= value << self.n
        self.n += numBits

    def getBitPosition(self):
        return self.n % 8

    def finish(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


class LzLeaf:
    """An Lz77Huffman preset by name (RLE_DYNAMIC, FULL_STATIC, ...)."""

    def __init__(self, name):
        self.name = name

    def decide(self, b, off, hl, dl):
        hist = bytes(b[off + max(0, hl - 32768):off + hl])
        data = bytes(b[off + hl:off + hl + dl])
        raw, nbits = O.deflate_chunks(hist, data, dl == 0, self.name, max(dl, 1), 32768 if hl else 0)
        val = int.from_bytes(raw, "little") & ((1 << nbits) - 1)
        val &= ~1                                  # written non-final; compressTo sets bfinal

        class D:
            def getBitLengths(self_):
                return [nbits] * 8

            def compressTo(self_, out, isFinal):
                v = val | (1 if isFinal else 0)
                done = 0
                while done < nbits:
                    k = min(16, nbits - done)
                    out.writeBits((v >> done) & ((1 << k) - 1), k)
                    done += k
        return D()


class UncLeaf:
    def decide(self, b, off, hl, dl):
        nb = max(-(-dl // 65535), 1)
        bits = [dl * 8 + nb * 40 + ((13 - i) % 8 - 5) for i in range(8)]
        data = bytes(b[off + hl:off + hl + dl])

        class D:
            def getBitLengths(self_):
                return bits

            def compressTo(self_, out, isFinal):
                i = 0
                while True:
                    n = min(dl - i, 65535)
                    out.writeBits(1 if isFinal and n == dl - i else 0, 1)
                    out.writeBits(0, 2)
                    out.writeBits(0, (8 - out.getBitPosition()) % 8)
                    out.writeBits(n, 16)
                    out.writeBits(n ^ 0xFFFF, 16)
                    for x in data[i:i + n]:
                        out.writeBits(x, 8)
                    i += n
                    if i >= dl:
                        break
        return D()


class Multi:
    def __init__(self, *subs):
        self.subs = subs

    def decide(self, b, off, hl, dl):
        bits, pick = [LONG_MAX] * 8, [None] * 8
        for st in self.subs:
            d = st.decide(b, off, hl, dl)
            for i, x in enumerate(d.getBitLengths()):
                if x < bits[i]:
                    bits[i], pick[i] = x, d

        class D:
            def getBitLengths(self_):
                return bits

            def compressTo(self_, out, isFinal):
                pick[out.getBitPosition()].compressTo(out, isFinal)
        return D()


class Split:
    def __init__(self, sub, m):
        self.sub, self.m = sub, m

    def decide(self, b, off, hl, dl, cur=None):
        cur = cur or self.sub.decide(b, off, hl, dl)
        seqs = [[cur]] * 8
        bits = list(cur.getBitLengths())
        h1 = (dl + 1) // 2
        h2 = dl - h1
        if min(h1, h2) > self.m:
            sp = [self.sub.decide(b, off, hl, h1), self.sub.decide(b, off, hl + h1, h2)]

            def tot(ds):
                t = 0
                for d in ds:
                    t += d.getBitLengths()[t % 8]
                return t
            if any(tot(sp) < bits[i] for i in range(8)):
                sp = [self.decide(b, off, hl, h1, sp[0]), self.decide(b, off, hl + h1, h2, sp[1])]
            for i in range(8):
                if tot(sp) < bits[i]:
                    bits[i], seqs[i] = tot(sp), sp

        class D:
            def getBitLengths(self_):
                return bits

            def compressTo(self_, out, isFinal):
                ds = seqs[out.getBitPosition()]
                for k, d in enumerate(ds):
                    d.compressTo(out, isFinal and k == len(ds) - 1)
        return D()


def stream(data, strategy, chunk=65536, hist_limit=32768):
    """DeflaterOutputStream(out, chunk, hist_limit, strategy) fed `data` then finished."""
    w = BitWriter()
    hist, pos, n = b"", 0, len(data)
    while True:
        k = min(chunk, n - pos)
        combined = hist + data[pos:pos + k]
        strategy.decide(combined, 0, len(hist), k).compressTo(w, pos + k == n)
        hist = combined[-hist_limit:] if hist_limit else b""
        pos += k
        if pos >= n:
            break
    return w.finish()
