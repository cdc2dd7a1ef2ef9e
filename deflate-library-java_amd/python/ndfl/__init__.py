"""ndfl -- MI355X-native DEFLATE codec, host-side mirror of io.nayuki.deflate.

The classes here mirror the reference's public API (same names, argument meaning and error
behaviour) on top of the C ABI in include/ndfl.h.  All codec work happens in libndfl.so's HIP
kernels; this module only buffers bytes, writes container headers and raises exceptions.

    DeflaterOutputStream   D/DeflaterOutputStream.java
    InflaterInputStream    D/InflaterInputStream.java
    DataFormatException    D/DataFormatException.java (with Reason)
    GzipMetadata           D/GzipMetadata.java
    GzipOutputStream       D/GzipOutputStream.java
    GzipInputStream        D/GzipInputStream.java
    ZlibOutputStream/ZlibInputStream/ZlibMetadata   D/Zlib*.java
"""
import ctypes
import enum
import io
import sys

from . import _lib
from ._lib import IN_DEVICE, OUT_DEVICE, DICT_DEFERRED, IN_PADDED, IN_PAD_BYTES, IN_PARTIAL, NEED_INPUT, NO_END, STRATEGIES, NdflError, check, load, reason_name

__all__ = ["Context", "Reason", "DataFormatException", "Lz77Huffman", "Uncompressed", "MultiStrategy", "BinarySplit", "DeflaterOutputStream", "InflaterInputStream", "BitOutputStream",
           "GzipMetadata", "GzipOutputStream", "GzipInputStream", "ZlibMetadata", "ZlibOutputStream",
           "ZlibInputStream", "Strategy", "default_context", "compress", "decompress", "crc32_combine"]


class Reason(enum.Enum):
    """DataFormatException.Reason (D/DataFormatException.java:61-83), same ordinal order."""
    UNEXPECTED_END_OF_STREAM = 0
    RESERVED_BLOCK_TYPE = 1
    UNCOMPRESSED_BLOCK_LENGTH_MISMATCH = 2
    HUFFMAN_CODE_UNDER_FULL = 3
    HUFFMAN_CODE_OVER_FULL = 4
    NO_PREVIOUS_CODE_LENGTH_TO_COPY = 5
    CODE_LENGTH_CODE_OVER_FULL = 6
    END_OF_BLOCK_CODE_ZERO_LENGTH = 7
    RESERVED_LENGTH_SYMBOL = 8
    RESERVED_DISTANCE_SYMBOL = 9
    LENGTH_ENCOUNTERED_WITH_EMPTY_DISTANCE_CODE = 10
    COPY_FROM_BEFORE_DICTIONARY_START = 11
    HEADER_CHECKSUM_MISMATCH = 12
    UNSUPPORTED_COMPRESSION_METHOD = 13
    DECOMPRESSED_CHECKSUM_MISMATCH = 14
    DECOMPRESSED_SIZE_MISMATCH = 15
    GZIP_INVALID_MAGIC_NUMBER = 16
    GZIP_RESERVED_FLAGS_SET = 17
    GZIP_UNSUPPORTED_OPERATING_SYSTEM = 18


class DataFormatException(Exception):
    """Unchecked in the reference (extends RuntimeException, D/DataFormatException.java:15): it is
    not made sticky by InflaterInputStream and not caught by the CLIs."""

    def __init__(self, reason, msg=None, symbol=-1):
        self.reason = reason
        if msg is None:
            msg = load().ndfl_error_string(reason.value + 1).decode()
            # the reference names the reserved symbol: "Reserved run length symbol: " + sym,
            # "Reserved distance symbol: " + sym (D/decomp/Open.java:516, 550, 659, 674)
            if symbol >= 0 and reason in (Reason.RESERVED_LENGTH_SYMBOL, Reason.RESERVED_DISTANCE_SYMBOL):
                msg += f": {symbol}"
        super().__init__(msg)

    def getReason(self):
        return self.reason


class Strategy(enum.Enum):
    """Lz77Huffman presets (D/comp/Lz77Huffman.java:298-305) and Uncompressed."""
    LITERAL_STATIC = 0
    LITERAL_DYNAMIC = 1
    RLE_STATIC = 2
    RLE_DYNAMIC = 3
    FULL_STATIC = 4
    FULL_DYNAMIC = 5
    UNCOMPRESSED = 6


class Lz77Huffman:
    """The Lz77Huffman record (D/comp/Lz77Huffman.java:20-39): greedy longest-match LZ77 over
    distances [searchMinimumDistance, searchMaximumDistance] with runs in [searchMinimumRunLength,
    searchMaximumRunLength], then static or dynamic Huffman codes.  Validation as :28-38
    (ValueError = IllegalArgumentException).  Presets as class attributes (:298-305)."""

    def __init__(self, useDynamicHuffmanCodes, searchMinimumRunLength, searchMaximumRunLength,
                 searchMinimumDistance, searchMaximumDistance):
        p = (searchMinimumRunLength, searchMaximumRunLength, searchMinimumDistance, searchMaximumDistance)
        mnr, mxr, mnd, mxd = p
        if not (p == (0, 0, 0, 0) or (3 <= mnr <= mxr <= 258 and 1 <= mnd <= mxd <= 32768)):
            raise ValueError("Invalid minimum/maximum run-length/distance")
        self.useDynamicHuffmanCodes = bool(useDynamicHuffmanCodes)
        self.params = p

    def __eq__(self, other):
        return isinstance(other, Lz77Huffman) and (self.useDynamicHuffmanCodes, self.params) == \
            (other.useDynamicHuffmanCodes, other.params)

    def __hash__(self):
        return hash((self.useDynamicHuffmanCodes, self.params))

    def __repr__(self):
        return f"Lz77Huffman({self.useDynamicHuffmanCodes}, {', '.join(map(str, self.params))})"

    def decide(self, b, off, historyLen, dataLen):
        """Strategy.decide (D/comp/Lz77Huffman.java:42-59), encoded on the GPU (ndfl_decide)."""
        return self._decide(b, off, historyLen, dataLen)

    def _decide(self, b, off, historyLen, dataLen, context=None):
        from .plugin import library_decide
        return library_decide(self, b, off, historyLen, dataLen, context)


Lz77Huffman.LITERAL_STATIC = Lz77Huffman(False, 0, 0, 0, 0)
Lz77Huffman.LITERAL_DYNAMIC = Lz77Huffman(True, 0, 0, 0, 0)
Lz77Huffman.RLE_STATIC = Lz77Huffman(False, 3, 258, 1, 1)
Lz77Huffman.RLE_DYNAMIC = Lz77Huffman(True, 3, 258, 1, 1)
Lz77Huffman.FULL_STATIC = Lz77Huffman(False, 3, 258, 1, 32768)
Lz77Huffman.FULL_DYNAMIC = Lz77Huffman(True, 3, 258, 1, 32768)


class _UncompressedType:
    """Uncompressed.SINGLETON (D/comp/Uncompressed.java:14-54): stored blocks of <= 65535 bytes."""

    def __repr__(self):
        return "Uncompressed.SINGLETON"

    def decide(self, b, off, historyLen, dataLen):
        """Strategy.decide (D/comp/Uncompressed.java:22-51)."""
        return self._decide(b, off, historyLen, dataLen)

    def _decide(self, b, off, historyLen, dataLen, context=None):
        from .plugin import library_decide
        return library_decide(self, b, off, historyLen, dataLen, context)


class Uncompressed:
    SINGLETON = _UncompressedType()


class MultiStrategy:
    """MultiStrategy(strats...) (D/comp/MultiStrategy.java:19-57): per chunk and output bit position,
    the first substrategy giving the fewest bits.  Substrategies: any Strategy (the library's
    classes, or a user object with decide()); a flat list of at most 8 Lz77Huffman / Uncompressed
    runs batched on the GPU (ndfl_deflate_chunks_multi), anything else per chunk (ndfl.plugin)."""

    def __init__(self, *strats):
        if strats is None or any(s is None for s in strats):
            raise TypeError("strategy")
        if len(strats) == 0:
            raise ValueError("Empty list of strategies")
        for st in strats:
            if not (isinstance(st, Strategy) or hasattr(st, "decide")):
                raise TypeError(f"not a strategy: {st!r}")
        self.substrategies = tuple(strats)

    def decide(self, b, off, historyLen, dataLen):
        return self._decide(b, off, historyLen, dataLen)

    def _decide(self, b, off, historyLen, dataLen, context=None):
        from .plugin import library_decide
        return library_decide(self, b, off, historyLen, dataLen, context)


class BinarySplit:
    """BinarySplit(strat, minBlockLen) (D/comp/BinarySplit.java:15-82): halve each chunk recursively
    while both halves exceed minBlockLen, keeping a split when it takes fewer bits.  Over an
    Lz77Huffman the whole stream is batched on the GPU (ndfl_deflate_chunks_binsplit); over any
    other Strategy it runs per chunk (ndfl.plugin: ndfl_decide for the library's classes)."""

    def __init__(self, strat, minBlockLen):
        if strat is None:
            raise TypeError("strat")
        if minBlockLen < 1:
            raise ValueError("Non-positive minimum block length")
        self.substrategy = strat
        self.minimumBlockLength = int(minBlockLen)

    def decide(self, b, off, historyLen, dataLen):
        return self._decide(b, off, historyLen, dataLen)

    def _decide(self, b, off, historyLen, dataLen, context=None):
        from .plugin import library_decide
        return library_decide(self, b, off, historyLen, dataLen, context)


def _desc(st):
    d = _lib.StrategyDesc()
    if isinstance(st, _UncompressedType):
        d.kind = _lib.KIND_UNCOMPRESSED
    else:
        d.kind = _lib.KIND_LZ77
        d.dynamic = int(st.useDynamicHuffmanCodes)
        d.min_run, d.max_run, d.min_dist, d.max_dist = st.params
    return d


def _ptr(obj):
    """(address, keepalive) of bytes-like / torch tensor."""
    if hasattr(obj, "data_ptr"):
        return obj.data_ptr(), obj
    if isinstance(obj, (bytes, bytearray, memoryview)):
        b = bytes(obj)
        buf = ctypes.create_string_buffer(b, max(1, len(b)))
        return ctypes.addressof(buf), buf
    raise TypeError(type(obj))


class Context:
    """One device context (HIP stream + device scratch).  Not reentrant.

    Stream ordering: unless set_stream() named a stream, every call that touches device memory
    runs on torch's current stream of this device when torch has initialised the GPU (so a
    tensor a torch kernel is still producing, or a block the caching allocator reuses, is ordered
    like any torch op), else after the device's default stream (the C ABI's own rule,
    include/ndfl.h)."""

    def __init__(self, device=0):
        L = load()
        h = ctypes.c_void_p()
        check(L.ndfl_ctx_create(ctypes.byref(h), device, 0), "ndfl_ctx_create")
        self._h = h
        self.device = device
        self._explicit_stream = False
        self._bound = None

    def _order(self):
        """Bind torch's current stream (see the class docstring) before a device call."""
        if self._explicit_stream:
            return
        torch = sys.modules.get("torch")
        if torch is None or not torch.cuda.is_initialized():
            return
        h = torch.cuda.current_stream(self.device).cuda_stream
        if h != self._bound:
            check(load().ndfl_ctx_set_stream(self._h, ctypes.c_void_p(h)))
            self._bound = h

    def close(self):
        if getattr(self, "_h", None):
            load().ndfl_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle):
        """Run this context's calls on the caller's HIP stream (None / 0: the default rule)."""
        check(load().ndfl_ctx_set_stream(self._h, ctypes.c_void_p(stream_handle)))
        self._explicit_stream = bool(stream_handle)
        self._bound = stream_handle

    def last_kernel_ms(self):
        return load().ndfl_ctx_last_kernel_ms(self._h)

    def timings(self):
        """{'deflate', 'inflate_find', 'inflate_count', 'inflate_emit', 'inflate_span'} in ms."""
        arr = (ctypes.c_double * 9)()
        load().ndfl_ctx_timings(self._h, arr, 9)
        keys = ["deflate", "inflate_find", "inflate_count", "inflate_emit", "inflate_span", "inflate_chains",
                "inflate_repairs", "inflate_candidates", "inflate_flat_chains"]
        return dict(zip(keys, list(arr)))

    # -- raw C-ABI wrappers ------------------------------------------------------------------
    def deflate_chunks_raw(self, hist_addr, hist_len, hist_limit, data_addr, n, chunk_len, strategy, final,
                           start_bitpos, out_addr, out_cap, flags, crc=None):
        L = load()
        self._order()
        endbits = ctypes.c_uint64(0)
        crcv = ctypes.c_uint32(crc if crc is not None else 0)
        crcp = ctypes.byref(crcv) if crc is not None else None
        if isinstance(strategy, BinarySplit):
            d = _desc(strategy.substrategy)
            r = L.ndfl_deflate_chunks_binsplit(self._h, hist_addr, hist_len, hist_limit, data_addr, n, chunk_len,
                                               ctypes.byref(d), strategy.minimumBlockLength, int(final), start_bitpos,
                                               out_addr, out_cap, ctypes.byref(endbits), crcp, flags)
            check(r, "ndfl_deflate_chunks_binsplit")
        elif isinstance(strategy, (MultiStrategy, _UncompressedType)):
            subs = strategy.substrategies if isinstance(strategy, MultiStrategy) else (strategy,)
            arr = (_lib.StrategyDesc * len(subs))(*[_desc(x) for x in subs])
            r = L.ndfl_deflate_chunks_multi(self._h, hist_addr, hist_len, hist_limit, data_addr, n, chunk_len, arr,
                                            len(subs), int(final), start_bitpos, out_addr, out_cap,
                                            ctypes.byref(endbits), crcp, flags)
            check(r, "ndfl_deflate_chunks_multi")
        elif isinstance(strategy, Lz77Huffman):
            r = L.ndfl_deflate_chunks_lz77(self._h, hist_addr, hist_len, hist_limit, data_addr, n, chunk_len,
                                           int(strategy.useDynamicHuffmanCodes), *strategy.params, int(final),
                                           start_bitpos, out_addr, out_cap, ctypes.byref(endbits), crcp, flags)
            check(r, "ndfl_deflate_chunks_lz77")
        else:
            r = L.ndfl_deflate_chunks(self._h, hist_addr, hist_len, hist_limit, data_addr, n, chunk_len,
                                      _strategy_id(strategy), int(final), start_bitpos, out_addr, out_cap,
                                      ctypes.byref(endbits), crcp, flags)
            check(r, "ndfl_deflate_chunks")
        return endbits.value, (crcv.value if crc is not None else None)

    def deflate(self, data, strategy=Strategy.RLE_DYNAMIC, chunk_len=65536, hist_limit=32768, with_crc=False):
        """Whole-stream compress of host bytes (DeflaterOutputStream write-all + finish)."""
        data = bytes(data)
        L = load()
        cap = L.ndfl_deflate_bound(len(data), chunk_len) + 16
        out = ctypes.create_string_buffer(cap)
        src = ctypes.create_string_buffer(data, max(1, len(data)))
        endbits, crc = self.deflate_chunks_raw(None, 0, hist_limit, ctypes.addressof(src), len(data), chunk_len,
                                               strategy, True, 0, ctypes.addressof(out), cap, 0,
                                               crc=0 if with_crc else None)
        comp = out.raw[:(endbits + 7) // 8]
        return (comp, crc) if with_crc else comp

    def inflate_raw(self, in_addr, in_len, out_addr, out_cap, flags):
        """Returns (code, out_len, consumed_bits); code = 0 / reason+1 / <0 error."""
        L = load()
        self._order()
        olen = ctypes.c_uint64(0)
        bits = ctypes.c_uint64(0)
        r = L.ndfl_inflate(self._h, in_addr, in_len, out_addr, out_cap, ctypes.byref(olen), ctypes.byref(bits),
                           flags)
        return r, olen.value, bits.value

    def inflate(self, data, out_cap=None):
        """Decode a whole raw DEFLATE stream held in host memory.  Returns (reason|None, bytes, bits)."""
        data = bytes(data)
        src = ctypes.create_string_buffer(data, max(1, len(data)))
        cap = out_cap if out_cap is not None else 4 * len(data) + 65536
        while True:
            out = ctypes.create_string_buffer(max(1, cap))
            r, olen, bits = self.inflate_raw(ctypes.addressof(src), len(data), ctypes.addressof(out), cap, 0)
            if r == _lib.E_CAPACITY and out_cap is None:
                cap = olen + 16
                continue
            check(r, "ndfl_inflate")
            reason = None if r == 0 else Reason(r - 1)
            return reason, out.raw[:olen], bits

    def error_symbol(self):
        """ndfl_ctx_error_symbol: the reserved symbol behind the last decode's RESERVED_LENGTH_SYMBOL /
        RESERVED_DISTANCE_SYMBOL (286/287, 30/31), or -1."""
        return load().ndfl_ctx_error_symbol(self._h)

    def data_format_error(self, code):
        """The DataFormatException of a decode that returned Reason+1 `code`, with the reference's
        message (the symbol appended where D/decomp/Open.java appends it)."""
        return DataFormatException(Reason(code - 1), symbol=self.error_symbol())

    def inflate_range_raw(self, in_addr, in_len, start_bit, end_bit, out_addr, dict_len, out_cap, flags):
        """ndfl_inflate_range: decode bits [start_bit, end_bit) into out_addr + dict_len, with the
        dict_len bytes at out_addr as the window.  Returns (code, out_len, consumed_bits)."""
        L = load()
        self._order()
        olen = ctypes.c_uint64(0)
        bits = ctypes.c_uint64(0)
        r = L.ndfl_inflate_range(self._h, in_addr, in_len, start_bit, NO_END if end_bit is None else end_bit,
                                 out_addr, dict_len, out_cap, ctypes.byref(olen), ctypes.byref(bits), flags)
        return r, olen.value, bits.value

    def inflate_sync_raw(self, in_addr, in_len, from_bit, window_bits, flags):
        """ndfl_inflate_sync: first confirmed block boundary at or past from_bit (None: none)."""
        self._order()
        v = ctypes.c_uint64(0)
        check(load().ndfl_inflate_sync(self._h, in_addr, in_len, from_bit, window_bits, ctypes.byref(v), flags),
              "ndfl_inflate_sync")
        return None if v.value == NO_END else v.value

    def inflate_headers_raw(self, in_addr, in_len, flags, survivors=False):
        """ndfl_inflate_headers (diagnostics): the decoder's chain starts, sorted; with survivors=True
        also the finder's survivors.  Returns (headers, stats[, survivors])."""
        L = load()
        self._order()
        n = ctypes.c_uint64(0)
        st = (ctypes.c_uint64 * 4)()
        check(L.ndfl_inflate_headers(self._h, in_addr, in_len, flags, None, 0, ctypes.byref(n), None, 0, st),
              "ndfl_inflate_headers")
        hs = (ctypes.c_uint64 * max(1, n.value))()
        ns = min(st[0], 2 * in_len + 65536) if survivors else 0
        sv = (ctypes.c_uint64 * max(1, ns))()
        check(L.ndfl_inflate_headers(self._h, in_addr, in_len, flags, hs, n.value, ctypes.byref(n),
                                     sv if ns else None, ns, st), "ndfl_inflate_headers")
        res = (list(hs[:n.value]), list(st))
        return res + (list(sv[:min(ns, st[0])]),) if survivors else res

    def inflate_headers(self, data, survivors=False):
        """inflate_headers_raw over a stream in host memory."""
        data = bytes(data)
        src = ctypes.create_string_buffer(data, max(1, len(data)))
        return self.inflate_headers_raw(ctypes.addressof(src), len(data), 0, survivors)

    def inflate_resolve(self):
        """Finish a DICT_DEFERRED range decode once the window is written; returns re-emitted chains."""
        self._order()
        n = ctypes.c_uint64(0)
        check(load().ndfl_inflate_resolve(self._h, ctypes.byref(n)), "ndfl_inflate_resolve")
        return n.value

    def inflate_tail_raw(self, tail_len, dst_addr):
        """ndfl_inflate_tail: the last tail_len output bytes of the pending DICT_DEFERRED decode (its
        window written) into device memory at dst_addr; False if a reference chain is too long
        (NDFL_E_UNSUPPORTED: resolve first)."""
        self._order()
        r = load().ndfl_inflate_tail(self._h, tail_len, ctypes.c_void_p(dst_addr))
        if r == _lib.E_UNSUPPORTED:
            return False
        check(r, "ndfl_inflate_tail")
        return True

    def inflate_tail_map_raw(self, tail_len, dst_addr):
        """ndfl_inflate_tail_map: the last tail_len output bytes of the pending DICT_DEFERRED decode
        as a map of its window (u32 per byte at dst_addr, device memory: window index, or
        TAIL_LITERAL | value); False if a reference chain is too long (NDFL_E_UNSUPPORTED)."""
        self._order()
        r = load().ndfl_inflate_tail_map(self._h, tail_len, ctypes.c_void_p(dst_addr))
        if r == _lib.E_UNSUPPORTED:
            return False
        check(r, "ndfl_inflate_tail_map")
        return True

    def bits_shift_raw(self, in_addr, nbits, shift, out_addr, out_cap):
        """ndfl_bits_shift on device buffers: in's first nbits bits placed at bit `shift` of out."""
        self._order()
        check(load().ndfl_bits_shift(self._h, in_addr, nbits, shift, out_addr, out_cap, IN_DEVICE | OUT_DEVICE),
              "ndfl_bits_shift")

    def crc32(self, data, crc=0, flags=0):
        self._order()
        addr, keep = _ptr(data)
        n = data.numel() * data.element_size() if hasattr(data, "numel") else len(data)
        v = ctypes.c_uint32(crc)
        check(load().ndfl_crc32(self._h, ctypes.byref(v), addr, n, flags), "ndfl_crc32")
        return v.value


    def adler32(self, data, adler=1, flags=0):
        self._order()
        addr, keep = _ptr(data)
        n = data.numel() * data.element_size() if hasattr(data, "numel") else len(data)
        v = ctypes.c_uint32(adler)
        check(load().ndfl_adler32(self._h, ctypes.byref(v), addr, n, flags), "ndfl_adler32")
        return v.value


def _ctx_default(context):
    return context if context is not None else default_context()


def _batchable(s):
    """Strategies the batched GPU calls take whole (ndfl_deflate_chunks / _lz77 / _multi /
    _binsplit); others go chunk by chunk through the plugin API."""
    if isinstance(s, (Strategy, str, int, Lz77Huffman, _UncompressedType)):
        return True
    if isinstance(s, MultiStrategy):
        return len(s.substrategies) <= 8 and all(isinstance(x, (Lz77Huffman, _UncompressedType))
                                                 for x in s.substrategies)
    if isinstance(s, BinarySplit):
        return isinstance(s.substrategy, Lz77Huffman)
    return False


def _strategy_id(s):
    if isinstance(s, (Lz77Huffman, MultiStrategy, _UncompressedType, BinarySplit)):
        return s
    if isinstance(s, Strategy):
        return s.value
    if isinstance(s, str):
        return STRATEGIES[s]
    return int(s)


def crc32_combine(a, b, len_b):
    return load().ndfl_crc32_combine(a, b, len_b)


_default = None


def default_context():
    global _default
    if _default is None:
        _default = Context(0)
    return _default


def compress(data, strategy=Strategy.RLE_DYNAMIC):
    return default_context().deflate(data, strategy)


def decompress(data):
    ctx = default_context()
    reason, out, _ = ctx.inflate(data)
    if reason is not None:
        raise ctx.data_format_error(reason.value + 1)
    return out


from .streams import (DeflaterOutputStream, InflaterInputStream, GzipMetadata, GzipOutputStream,  # noqa: E402
                      GzipInputStream, ZlibMetadata, ZlibOutputStream, ZlibInputStream)
from .plugin import BitOutputStream  # noqa: E402
