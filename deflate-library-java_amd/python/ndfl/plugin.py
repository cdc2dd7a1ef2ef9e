"""The compressor plugin API of the reference (D/comp/Strategy.java:14, D/comp/Decision.java:16-19,
D/comp/BitOutputStream.java:16-19) on the GPU encoders.

    Strategy        any object with decide(b, off, historyLen, dataLen) -> Decision
    Decision        getBitLengths() -> 8 ints (bits when the block starts at bit position i mod 8);
                    compressTo(out: BitOutputStream, isFinal)
    BitOutputStream writeBits(value, numBits) (LSB first, 0 <= numBits <= 31), getBitPosition()

The library's own strategies (Lz77Huffman, Uncompressed, MultiStrategy, BinarySplit) decide on the
GPU through ndfl_decide / ndfl_compress_to (include/ndfl.h) whenever their whole tree is built of
them; a tree holding a user strategy is composed here, with the reference's own rules
(D/comp/MultiStrategy.java:31-57, D/comp/BinarySplit.java:36-82), so user strategies mix freely
with GPU ones.  DeflaterOutputStream takes this per-chunk path for any strategy the batched GPU
calls do not cover.
"""
import ctypes

from . import _lib
from ._lib import check, load


class BitOutputStream:
    """D/comp/BitOutputStream.java (interface)."""

    def writeBits(self, value, numBits):
        raise NotImplementedError

    def getBitPosition(self):
        raise NotImplementedError


class BitBuffer(BitOutputStream):
    """DeflaterOutputStream.BitOut (D/DeflaterOutputStream.java:141-171) into a bytearray: LSB-first
    bit packing; `pending` holds the partial last byte.  take_bytes() hands out the whole bytes."""

    def __init__(self, bitpos=0, partial=0):
        self.buf = bytearray()
        self.nbits = bitpos          # bits in buf + the partial byte
        self.partial = partial & ((1 << bitpos) - 1) if bitpos else 0

    def writeBits(self, value, numBits):
        if not (0 <= numBits <= 31) or value >> numBits:
            raise ValueError("writeBits")
        acc = self.partial | (value << (self.nbits & 7))
        n = (self.nbits & 7) + numBits
        while n >= 8:
            self.buf.append(acc & 0xFF)
            acc >>= 8
            n -= 8
        self.partial = acc
        self.nbits += numBits

    def getBitPosition(self):
        return self.nbits & 7

    def _append_bytes(self, data, nbits):
        """Append nbits bits laid out LSB-first from bit getBitPosition() of data[0] (the lower
        bits of data[0] are ignored): the output of ndfl_compress_to at that start position."""
        p = self.nbits & 7
        if nbits == 0:
            return
        b = bytearray(data[:(p + nbits + 7) // 8])
        b[0] = (b[0] & ~((1 << p) - 1) & 0xFF) | self.partial
        end = p + nbits
        whole = end // 8
        self.buf += b[:whole]
        self.partial = b[whole] & ((1 << (end & 7)) - 1) if end & 7 else 0
        self.nbits += nbits

    def take_bytes(self):
        out = bytes(self.buf)
        self.buf = bytearray()
        return out


def _node(kind, dynamic=0, params=(0, 0, 0, 0), first_child=0, n_children=0, min_block_len=0):
    n = _lib.StrategyNode()
    n.kind = kind
    n.dynamic = dynamic
    n.min_run, n.max_run, n.min_dist, n.max_dist = params
    n.first_child, n.n_children, n.min_block_len = first_child, n_children, min_block_len
    return n


def native_tree(strategy):
    """ndfl_strategy_node array of a strategy built only of the library's classes (root at 0), or
    None when the tree holds a user strategy."""
    from . import Lz77Huffman, MultiStrategy, BinarySplit, Strategy, Uncompressed, _UncompressedType
    nodes = []

    def add(st):
        if isinstance(st, Strategy):
            st = Uncompressed.SINGLETON if st == Strategy.UNCOMPRESSED else getattr(Lz77Huffman, st.name)
        idx = len(nodes)
        nodes.append(None)
        if isinstance(st, Lz77Huffman):
            nodes[idx] = _node(_lib.KIND_LZ77, int(st.useDynamicHuffmanCodes), st.params)
        elif isinstance(st, _UncompressedType):
            nodes[idx] = _node(_lib.KIND_UNCOMPRESSED)
        elif isinstance(st, MultiStrategy):
            # children must be contiguous: reserve their slots first, then fill subtrees after them
            first = len(nodes)
            nodes.extend([None] * len(st.substrategies))
            kids = []
            for k, sub in enumerate(st.substrategies):
                sub_idx = add(sub)
                if sub_idx is None:
                    return None
                kids.append(sub_idx)
            for k, sub_idx in enumerate(kids):          # slot k: a copy of the child's node
                nodes[first + k] = nodes[sub_idx]
            nodes[idx] = _node(_lib.KIND_MULTI, first_child=first, n_children=len(kids))
        elif isinstance(st, BinarySplit):
            sub_idx = add(st.substrategy)
            if sub_idx is None:
                return None
            nodes[idx] = _node(_lib.KIND_BINSPLIT, first_child=sub_idx, min_block_len=st.minimumBlockLength)
        else:
            return None
        return idx

    if add(strategy) is None:
        return None
    return (_lib.StrategyNode * len(nodes))(*nodes)


class GpuDecision:
    """A Decision computed by ndfl_decide (GPU encodes of the Lz77Huffman leaves)."""

    def __init__(self, ctx, handle, bit_lengths, keep):
        self._ctx, self._h, self._bits, self._keep = ctx, handle, bit_lengths, keep

    def getBitLengths(self):
        return list(self._bits)

    def compressTo(self, out, isFinal):
        p = out.getBitPosition()
        # (BinarySplit's lengths index its halves from position 0, so the bits written at p may
        # exceed the reported length by the halves' stored-block padding)
        cap = max(self._bits) // 8 + 4096
        while True:
            buf = ctypes.create_string_buffer(cap)
            end = ctypes.c_uint64(0)
            r = load().ndfl_compress_to(self._ctx._h, self._h, int(bool(isFinal)), p, buf, cap, ctypes.byref(end))
            if r == _lib.E_CAPACITY:
                cap *= 2
                continue
            check(r, "ndfl_compress_to")
            break
        nbits = end.value - p
        if isinstance(out, BitBuffer):
            out._append_bytes(buf.raw, nbits)
            return
        # any BitOutputStream: feed the bits from position p on in pieces of <= 24
        v = int.from_bytes(buf.raw[:(end.value + 7) // 8], "little") >> p
        done = 0
        while done < nbits:
            k = min(24, nbits - done)
            out.writeBits((v >> done) & ((1 << k) - 1), k)
            done += k

    def __del__(self):
        try:
            if self._h:
                load().ndfl_decision_free(self._h)
                self._h = None
        except Exception:
            pass


def gpu_decide(ctx, nodes, b, off, historyLen, dataLen):
    """Strategy.decide for a native tree: ndfl_decide over b[off : off + historyLen + dataLen]."""
    mv = bytes(b[off:off + historyLen + dataLen])
    buf = ctypes.create_string_buffer(mv, max(1, len(mv)))
    bits = (ctypes.c_uint64 * 8)()
    h = ctypes.c_void_p()
    check(load().ndfl_decide(ctx._h, nodes, len(nodes), 0, buf, 0, historyLen, dataLen, bits, ctypes.byref(h)),
          "ndfl_decide")
    return GpuDecision(ctx, h, list(bits), buf)


class _Composed:
    """A Decision composed on the host (a MultiStrategy / BinarySplit holding user strategies)."""

    def __init__(self, bit_lengths, chooser):
        self._bits = bit_lengths
        self._choose = chooser

    def getBitLengths(self):
        return list(self._bits)

    def compressTo(self, out, isFinal):
        decs = self._choose(out.getBitPosition())
        for i, d in enumerate(decs):
            d.compressTo(out, isFinal and i == len(decs) - 1)


LONG_MAX = (1 << 63) - 1


def compose_multi(subs, b, off, historyLen, dataLen, decide):
    """MultiStrategy.decide (D/comp/MultiStrategy.java:31-57)."""
    bits = [LONG_MAX] * 8
    pick = [None] * 8
    for st in subs:
        dec = decide(st, b, off, historyLen, dataLen)
        bl = dec.getBitLengths()
        for i in range(8):
            if bl[i] < bits[i]:
                bits[i] = bl[i]
                pick[i] = dec
    if any(p is None for p in pick):
        raise TypeError("subdecision")
    return _Composed(bits, lambda p: [pick[p]])


def compose_split(sub, m, b, off, historyLen, dataLen, decide, cur=None):
    """BinarySplit.decide (D/comp/BinarySplit.java:36-82), including its accumulation that indexes
    each half's lengths from position 0."""
    if cur is None:
        cur = decide(sub, b, off, historyLen, dataLen)
    seqs = [[cur]] * 8
    bits = list(cur.getBitLengths())
    h1 = (dataLen + 1) // 2
    h2 = dataLen - h1
    if min(h1, h2) > m:
        split = [decide(sub, b, off, historyLen, h1), decide(sub, b, off, historyLen + h1, h2)]

        def total(decs):
            bl = 0
            for d in decs:
                bl += d.getBitLengths()[bl % 8]
            return bl
        if any(total(split) < bits[i] for i in range(8)):
            split = [compose_split(sub, m, b, off, historyLen, h1, decide, split[0]),
                     compose_split(sub, m, b, off, historyLen + h1, h2, decide, split[1])]
        for i in range(8):
            t = total(split)
            if t < bits[i]:
                bits[i] = t
                seqs[i] = split
    return _Composed(bits, lambda p: seqs[p])


def decide_any(st, b, off, historyLen, dataLen, context=None):
    """Strategy.decide of any strategy: the library's classes (GPU), Strategy enum members, or a
    user object with decide()."""
    from . import Strategy, _ctx_default
    if isinstance(st, Strategy):
        nodes = native_tree(st)
        return gpu_decide(_ctx_default(context), nodes, b, off, historyLen, dataLen)
    if hasattr(st, "_decide"):
        return st._decide(b, off, historyLen, dataLen, context)
    return st.decide(b, off, historyLen, dataLen)


def library_decide(st, b, off, historyLen, dataLen, context=None):
    """decide() of the library's strategy classes: one ndfl_decide for a native tree, else the
    reference's composition over the children (some of which are user strategies)."""
    from . import MultiStrategy, BinarySplit, _ctx_default
    nodes = native_tree(st)
    if nodes is not None:
        return gpu_decide(_ctx_default(context), nodes, b, off, historyLen, dataLen)
    dec = lambda s2, *a: decide_any(s2, *a, context=context)  # noqa: E731
    if isinstance(st, MultiStrategy):
        return compose_multi(st.substrategies, b, off, historyLen, dataLen, dec)
    if isinstance(st, BinarySplit):
        return compose_split(st.substrategy, st.minimumBlockLength, b, off, historyLen, dataLen, dec)
    raise TypeError(f"not a strategy: {st!r}")
