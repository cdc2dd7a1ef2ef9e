"""ctypes binding of oracle/liboracle.so (the CPU parity checker).  Test infrastructure only."""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None

REASONS = [
    "UNEXPECTED_END_OF_STREAM", "RESERVED_BLOCK_TYPE", "UNCOMPRESSED_BLOCK_LENGTH_MISMATCH",
    "HUFFMAN_CODE_UNDER_FULL", "HUFFMAN_CODE_OVER_FULL", "NO_PREVIOUS_CODE_LENGTH_TO_COPY",
    "CODE_LENGTH_CODE_OVER_FULL", "END_OF_BLOCK_CODE_ZERO_LENGTH", "RESERVED_LENGTH_SYMBOL",
    "RESERVED_DISTANCE_SYMBOL", "LENGTH_ENCOUNTERED_WITH_EMPTY_DISTANCE_CODE",
    "COPY_FROM_BEFORE_DICTIONARY_START", "HEADER_CHECKSUM_MISMATCH", "UNSUPPORTED_COMPRESSION_METHOD",
    "DECOMPRESSED_CHECKSUM_MISMATCH", "DECOMPRESSED_SIZE_MISMATCH", "GZIP_INVALID_MAGIC_NUMBER",
    "GZIP_RESERVED_FLAGS_SET", "GZIP_UNSUPPORTED_OPERATING_SYSTEM",
]

STRATEGIES = ["LITERAL_STATIC", "LITERAL_DYNAMIC", "RLE_STATIC", "RLE_DYNAMIC",
              "FULL_STATIC", "FULL_DYNAMIC", "UNCOMPRESSED"]


def reason_name(code):
    if code == 0:
        return None
    if 1 <= code <= len(REASONS):
        return REASONS[code - 1]
    return f"ERR{code}"


class GzipMeta(ctypes.Structure):
    _fields_ = [
        ("is_text", ctypes.c_int32), ("has_mtime", ctypes.c_int32), ("mtime", ctypes.c_uint32),
        ("extra_flags", ctypes.c_int32), ("os", ctypes.c_int32),
        ("has_extra", ctypes.c_int32), ("extra_len", ctypes.c_uint32), ("extra", ctypes.c_void_p),
        ("has_name", ctypes.c_int32), ("name", ctypes.c_char_p),
        ("has_comment", ctypes.c_int32), ("comment", ctypes.c_char_p),
        ("has_header_crc", ctypes.c_int32),
    ]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        src = os.path.join(ORACLE_DIR, "ndfl_oracle.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(path)
        u8p = ctypes.c_void_p
        L.or_deflate.restype = ctypes.c_int64
        L.or_deflate.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                 ctypes.c_int, u8p, ctypes.c_uint64]
        L.or_deflate_lz.restype = ctypes.c_int64
        L.or_deflate_lz.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    u8p, ctypes.c_uint64]
        L.or_deflate_multi.restype = ctypes.c_int64
        L.or_deflate_multi.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_uint32, u8p, ctypes.c_uint64]
        L.or_deflate_binsplit.restype = ctypes.c_int64
        L.or_deflate_binsplit.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_int32, u8p, ctypes.c_uint64]
        L.or_deflate_block_bits.restype = ctypes.c_int64
        L.or_deflate_block_bits.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
        L.or_deflate_mixed.restype = ctypes.c_int64
        L.or_deflate_mixed.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint32,
                                       u8p, ctypes.c_uint64]
        L.or_inflate.restype = ctypes.c_int
        L.or_inflate.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_uint64,
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.or_deflate_chunks.restype = ctypes.c_int64
        L.or_deflate_chunks.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_int, ctypes.c_int, u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.or_inflate_range.restype = ctypes.c_int
        L.or_inflate_range.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_uint64,
                                       u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint64)]
        L.or_scan_headers.restype = ctypes.c_int64
        L.or_scan_headers.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
        L.or_crc32.restype = ctypes.c_uint32
        L.or_crc32.argtypes = [ctypes.c_uint32, u8p, ctypes.c_uint64]
        L.or_adler32.restype = ctypes.c_uint32
        L.or_adler32.argtypes = [ctypes.c_uint32, u8p, ctypes.c_uint64]
        L.or_gzip_compress.restype = ctypes.c_int64
        L.or_gzip_compress.argtypes = [u8p, ctypes.c_uint64, ctypes.POINTER(GzipMeta), u8p, ctypes.c_uint64]
        L.or_gunzip.restype = ctypes.c_int
        L.or_gunzip.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.POINTER(GzipMeta), ctypes.POINTER(ctypes.c_uint64)]
        L.or_zlib_compress.restype = ctypes.c_int64
        L.or_zlib_compress.argtypes = [u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_uint64]
        L.or_zlib_decompress.restype = ctypes.c_int
        L.or_zlib_decompress.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.or_error_symbol.restype = ctypes.c_int
        L.or_error_symbol.argtypes = []
        _LIB = L
    return _LIB


def error_symbol():
    """The reserved symbol of this thread's last RESERVED_LENGTH_SYMBOL / RESERVED_DISTANCE_SYMBOL
    decode error (the suffix of the reference's message, D/decomp/Open.java:516, 550), else -1."""
    return lib().or_error_symbol()


def _buf(data):
    b = bytes(data)
    return ctypes.create_string_buffer(b, max(1, len(b))), len(b)


def deflate_bound(n, chunk_len=65536):
    return n + n // 4 + 4096 + (n // min(chunk_len, 65535) + 1) * 600


def deflate(data, strategy="RLE_DYNAMIC", chunk_len=65536, hist_limit=32768, brute=False):
    src, n = _buf(data)
    cap = deflate_bound(n, chunk_len)
    out = ctypes.create_string_buffer(cap)
    r = lib().or_deflate(src, n, chunk_len, hist_limit, STRATEGIES.index(strategy), int(brute), out, cap)
    if r < 0:
        raise ValueError(f"or_deflate failed: {r}")
    return out.raw[:r]


def deflate_lz(data, dynamic, min_run, max_run, min_dist, max_dist, chunk_len=65536, hist_limit=32768, brute=False):
    src, n = _buf(data)
    cap = deflate_bound(n, chunk_len) * 2
    out = ctypes.create_string_buffer(cap)
    r = lib().or_deflate_lz(src, n, chunk_len, hist_limit, int(dynamic), min_run, max_run, min_dist, max_dist,
                            int(brute), out, cap)
    if r < 0:
        raise ValueError(f"or_deflate_lz failed: {r}")
    return out.raw[:r]


def deflate_multi(data, subs, chunk_len=65536, hist_limit=32768):
    """MultiStrategy(subs...): each sub is "UNCOMPRESSED" or (dynamic, minRun, maxRun, minDist, maxDist)."""
    src, n = _buf(data)
    flat = []
    for st in subs:
        flat += [1, 0, 0, 0, 0, 0] if st == "UNCOMPRESSED" else [0] + [int(x) for x in st]
    arr = (ctypes.c_int32 * len(flat))(*flat)
    cap = deflate_bound(n, chunk_len) * 2
    out = ctypes.create_string_buffer(cap)
    r = lib().or_deflate_multi(src, n, chunk_len, hist_limit, arr, len(subs), out, cap)
    if r < 0:
        raise ValueError(f"or_deflate_multi failed: {r}")
    return out.raw[:r]


def deflate_binsplit(data, sub, min_block_len, chunk_len=65536, hist_limit=32768):
    """BinarySplit(sub, minBlockLen): sub is "UNCOMPRESSED" or (dynamic, minRun, maxRun, minDist, maxDist)."""
    src, n = _buf(data)
    flat = [1, 0, 0, 0, 0, 0] if sub == "UNCOMPRESSED" else [0] + [int(x) for x in sub]
    arr = (ctypes.c_int32 * 6)(*flat)
    cap = deflate_bound(n, chunk_len) * 2 + 4096
    out = ctypes.create_string_buffer(cap)
    r = lib().or_deflate_binsplit(src, n, chunk_len, hist_limit, arr, min_block_len, out, cap)
    if r < 0:
        raise ValueError(f"or_deflate_binsplit failed: {r}")
    return out.raw[:r]


def deflate_mixed(data, strategies, chunk_len=65535, hist_limit=32768):
    """Fixture generator: chunk i encoded with strategies[i % len]."""
    src, n = _buf(data)
    cap = deflate_bound(n, chunk_len) * 2
    out = ctypes.create_string_buffer(cap)
    st = (ctypes.c_int8 * len(strategies))(*[STRATEGIES.index(s) for s in strategies])
    r = lib().or_deflate_mixed(src, n, chunk_len, hist_limit, st, len(strategies), out, cap)
    if r < 0:
        raise ValueError(f"or_deflate_mixed failed: {r}")
    return out.raw[:r]


def deflate_chunks(hist, data, final, strategy="RLE_DYNAMIC", chunk_len=65536, hist_limit=32768):
    """ndfl_deflate_chunks semantics on the CPU: returns (bytes, nbits), stream starting at bit 0."""
    h, hn = _buf(hist)
    src, n = _buf(data)
    cap = deflate_bound(n, chunk_len)
    out = ctypes.create_string_buffer(cap)
    bits = ctypes.c_uint64(0)
    r = lib().or_deflate_chunks(h, hn, src, n, chunk_len, hist_limit, STRATEGIES.index(strategy), int(final), out, cap,
                                ctypes.byref(bits))
    if r < 0:
        raise ValueError(f"or_deflate_chunks failed: {r}")
    return out.raw[:r], bits.value


def block_bits(data, strategy="RLE_DYNAMIC", chunk_len=65536, hist_limit=32768):
    src, n = _buf(data)
    nchunks = max(1, -(-n // chunk_len))
    arr = (ctypes.c_uint64 * nchunks)()
    r = lib().or_deflate_block_bits(src, n, chunk_len, hist_limit, STRATEGIES.index(strategy), arr, nchunks)
    assert r == nchunks, (r, nchunks)
    return list(arr)


def inflate(data, out_cap=None):
    """Returns (reason_name_or_None, output_bytes, consumed_bits)."""
    src, n = _buf(data)
    cap = out_cap if out_cap is not None else 4 * n + 65536
    while True:
        out = ctypes.create_string_buffer(max(1, cap))
        olen = ctypes.c_uint64(0)
        bits = ctypes.c_uint64(0)
        r = lib().or_inflate(src, n, out, cap, ctypes.byref(olen), ctypes.byref(bits))
        if r == -1 and out_cap is None and cap < 1100 * n + 65536:
            cap *= 8
            continue
        if r < 0:
            raise ValueError(f"or_inflate error {r}")
        return reason_name(r), out.raw[:olen.value], bits.value


def inflate_range(data, start_bit=0, end_bit=None, dictionary=b"", out_cap=None):
    """Range decode (multi-GPU shard): start at start_bit with `dictionary` as preceding output, stop
    at the block boundary == end_bit (None: after the final block).  Returns like inflate()."""
    src, n = _buf(data)
    d, dn = _buf(dictionary)
    cap = out_cap if out_cap is not None else 4 * n + 65536
    while True:
        out = ctypes.create_string_buffer(max(1, cap))
        olen = ctypes.c_uint64(0)
        bits = ctypes.c_uint64(0)
        r = lib().or_inflate_range(src, n, start_bit, (1 << 64) - 1 if end_bit is None else end_bit, d, dn, out,
                                   cap, ctypes.byref(olen), ctypes.byref(bits))
        if r == -1 and out_cap is None and cap < 1100 * n + 65536:
            cap *= 8
            continue
        if r < 0:
            raise ValueError(f"or_inflate_range error {r}")
        return reason_name(r), out.raw[:olen.value], bits.value


def scan_headers(data, lo=0, hi=None):
    """The GPU decoder's chain starts in `data` (or_scan_headers): sorted bit positions."""
    L = lib()
    hi = len(data) * 8 if hi is None else hi
    b, nb = _buf(data)
    n = L.or_scan_headers(b, nb, lo, hi, None, 0)
    arr = (ctypes.c_uint64 * max(n, 1))()
    L.or_scan_headers(b, nb, lo, hi, arr, n)
    return list(arr[:n])


def crc32(data, crc=0):
    src, n = _buf(data)
    return lib().or_crc32(crc, src, n)


def adler32(data, adler=1):
    src, n = _buf(data)
    return lib().or_adler32(adler, src, n)


def gzip_compress(data, name=None, mtime=0, os_=3, header_crc=True, text=False, comment=None, extra=None,
                  extra_flags=0):
    m = GzipMeta()
    m.is_text = int(text)
    m.has_mtime = int(mtime != 0)
    m.mtime = mtime
    m.extra_flags = extra_flags
    m.os = os_
    keep = []
    if extra is not None:
        eb = ctypes.create_string_buffer(bytes(extra), max(1, len(extra)))
        keep.append(eb)
        m.has_extra, m.extra_len, m.extra = 1, len(extra), ctypes.cast(eb, ctypes.c_void_p)
    if name is not None:
        m.has_name, m.name = 1, name
    if comment is not None:
        m.has_comment, m.comment = 1, comment
    m.has_header_crc = int(header_crc)
    src, n = _buf(data)
    cap = deflate_bound(n) + 1024 + (len(name) if name else 0) + (len(comment) if comment else 0) + (len(extra) if extra else 0)
    out = ctypes.create_string_buffer(cap)
    r = lib().or_gzip_compress(src, n, ctypes.byref(m), out, cap)
    if r < 0:
        raise ValueError(f"or_gzip_compress failed {r}")
    return out.raw[:r]


def gunzip(data, out_cap=None):
    """Returns (reason_or_None, output, header_dict, member_end)."""
    src, n = _buf(data)
    cap = out_cap if out_cap is not None else 4 * n + (2 << 20)
    out = ctypes.create_string_buffer(cap)
    olen = ctypes.c_uint64(0)
    h = GzipMeta()
    end = ctypes.c_uint64(0)
    r = lib().or_gunzip(src, n, out, cap, ctypes.byref(olen), ctypes.byref(h), ctypes.byref(end))
    hd = {"is_text": bool(h.is_text), "mtime": h.mtime if h.has_mtime else None, "extra_flags": h.extra_flags,
          "os": h.os, "has_header_crc": bool(h.has_header_crc)}
    return reason_name(r) if r >= 0 else f"ERR{r}", out.raw[:olen.value], hd, end.value


def zlib_compress(data, cinfo=7, level=2):
    src, n = _buf(data)
    cap = deflate_bound(n) + 64
    out = ctypes.create_string_buffer(cap)
    r = lib().or_zlib_compress(src, n, cinfo, level, out, cap)
    if r < 0:
        raise ValueError(f"or_zlib_compress failed {r}")
    return out.raw[:r]


def zlib_decompress(data, out_cap=None):
    src, n = _buf(data)
    cap = out_cap if out_cap is not None else 4 * n + (2 << 20)
    out = ctypes.create_string_buffer(cap)
    olen = ctypes.c_uint64(0)
    r = lib().or_zlib_decompress(src, n, out, cap, ctypes.byref(olen))
    return (reason_name(r) if r >= 0 else f"ERR{r}"), out.raw[:olen.value]


def bits_to_bytes(bits, pad_mode=0, rng=None):
    """StringInputStream semantics (T/StringInputStream.java:40-47): each 8-char group, first
    char = least significant bit.  Pads to a byte multiple with 0s, 1s or random bits as the
    reference harness does (T/InflaterInputStreamTest.java:523-531)."""
    bits = bits.replace(" ", "")
    while len(bits) % 8:
        if pad_mode == 0:
            bits += "0"
        elif pad_mode == 1:
            bits += "1"
        else:
            bits += str(rng.randrange(2))
    if not bits:
        return b""
    return int(bits[::-1], 2).to_bytes(len(bits) // 8, "little")
