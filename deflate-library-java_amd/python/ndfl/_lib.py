"""ctypes binding of libndfl.so (include/ndfl.h).  Fails loudly if the HIP library is missing:
there is no CPU fallback on the product path."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(os.path.dirname(_HERE))          # deflate-library-java_amd/
LIB_PATH = os.environ.get("NDFL_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libndfl.so")

IN_DEVICE = 1
OUT_DEVICE = 2
DICT_DEFERRED = 4
IN_PADDED = 8          # NDFL_IN_PADDED: device input read in place (aligned, IN_PAD_BYTES zeros after)
IN_PAD_BYTES = 256
IN_PARTIAL = 16        # NDFL_IN_PARTIAL: the input is a prefix of the stream
NEED_INPUT = 64        # NDFL_NEED_INPUT: a partial-input decode stopped at a block boundary
NO_END = (1 << 64) - 1
TAIL_LITERAL = 0x80000000   # NDFL_TAIL_LITERAL: a window-map entry that holds a byte value

STRATEGIES = {"LITERAL_STATIC": 0, "LITERAL_DYNAMIC": 1, "RLE_STATIC": 2, "RLE_DYNAMIC": 3,
              "FULL_STATIC": 4, "FULL_DYNAMIC": 5, "UNCOMPRESSED": 6}

REASONS = [
    "UNEXPECTED_END_OF_STREAM", "RESERVED_BLOCK_TYPE", "UNCOMPRESSED_BLOCK_LENGTH_MISMATCH",
    "HUFFMAN_CODE_UNDER_FULL", "HUFFMAN_CODE_OVER_FULL", "NO_PREVIOUS_CODE_LENGTH_TO_COPY",
    "CODE_LENGTH_CODE_OVER_FULL", "END_OF_BLOCK_CODE_ZERO_LENGTH", "RESERVED_LENGTH_SYMBOL",
    "RESERVED_DISTANCE_SYMBOL", "LENGTH_ENCOUNTERED_WITH_EMPTY_DISTANCE_CODE",
    "COPY_FROM_BEFORE_DICTIONARY_START", "HEADER_CHECKSUM_MISMATCH", "UNSUPPORTED_COMPRESSION_METHOD",
    "DECOMPRESSED_CHECKSUM_MISMATCH", "DECOMPRESSED_SIZE_MISMATCH", "GZIP_INVALID_MAGIC_NUMBER",
    "GZIP_RESERVED_FLAGS_SET", "GZIP_UNSUPPORTED_OPERATING_SYSTEM",
]

E_ARG, E_UNSUPPORTED, E_CAPACITY, E_DEVICE, E_STATE, E_INTERNAL = -1, -2, -3, -4, -5, -6

# Every symbol include/ndfl.h declares (checked by tests/test_capi_symbols.py).
EXPORTS = ["ndfl_abi_version", "ndfl_error_string", "ndfl_ctx_create", "ndfl_ctx_destroy",
           "ndfl_ctx_set_stream", "ndfl_ctx_last_kernel_ms", "ndfl_ctx_timings", "ndfl_deflate_chunks",
           "ndfl_deflate_chunks_lz77", "ndfl_deflate_chunks_multi", "ndfl_deflate_chunks_binsplit",
           "ndfl_deflate_bound",
           "ndfl_inflate", "ndfl_inflate_range", "ndfl_inflate_resolve", "ndfl_bits_shift", "ndfl_crc32", "ndfl_adler32",
           "ndfl_crc32_combine", "ndfl_decide", "ndfl_compress_to", "ndfl_decision_free", "ndfl_inflate_sync",
           "ndfl_inflate_tail", "ndfl_inflate_headers", "ndfl_inflate_tail_map", "ndfl_ctx_error_symbol"]

KIND_LZ77, KIND_UNCOMPRESSED = 0, 1


KIND_MULTI, KIND_BINSPLIT = 2, 3


class StrategyNode(ctypes.Structure):
    """ndfl_strategy_node (include/ndfl.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("dynamic", ctypes.c_int32), ("min_run", ctypes.c_int32),
                ("max_run", ctypes.c_int32), ("min_dist", ctypes.c_int32), ("max_dist", ctypes.c_int32),
                ("first_child", ctypes.c_int32), ("n_children", ctypes.c_int32), ("min_block_len", ctypes.c_int32)]


class StrategyDesc(ctypes.Structure):
    """ndfl_strategy_desc (include/ndfl.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("dynamic", ctypes.c_int32), ("min_run", ctypes.c_int32),
                ("max_run", ctypes.c_int32), ("min_dist", ctypes.c_int32), ("max_dist", ctypes.c_int32)]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libndfl.so not built ({LIB_PATH}); run `make -C deflate-library-java_amd`")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.ndfl_abi_version.restype = u32
    L.ndfl_error_string.restype = ctypes.c_char_p
    L.ndfl_error_string.argtypes = [i32]
    L.ndfl_ctx_create.argtypes = [ctypes.POINTER(vp), i32, u32]
    L.ndfl_ctx_destroy.argtypes = [vp]
    L.ndfl_ctx_set_stream.argtypes = [vp, vp]
    L.ndfl_ctx_last_kernel_ms.restype = ctypes.c_double
    L.ndfl_ctx_last_kernel_ms.argtypes = [vp]
    L.ndfl_ctx_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i32]
    L.ndfl_ctx_error_symbol.argtypes = [vp]
    L.ndfl_deflate_chunks.argtypes = [vp, vp, u32, u32, vp, u64, u32, i32, i32, u32, vp, u64,
                                      ctypes.POINTER(u64), ctypes.POINTER(u32), u32]
    L.ndfl_deflate_chunks_lz77.argtypes = [vp, vp, u32, u32, vp, u64, u32, i32, i32, i32, i32, i32, i32, u32, vp,
                                           u64, ctypes.POINTER(u64), ctypes.POINTER(u32), u32]
    L.ndfl_deflate_chunks_multi.argtypes = [vp, vp, u32, u32, vp, u64, u32, ctypes.POINTER(StrategyDesc), u32, i32,
                                            u32, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u32), u32]
    L.ndfl_deflate_chunks_binsplit.argtypes = [vp, vp, u32, u32, vp, u64, u32, ctypes.POINTER(StrategyDesc), i32,
                                               i32, u32, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u32), u32]
    L.ndfl_deflate_bound.restype = u64
    L.ndfl_deflate_bound.argtypes = [u64, u32]
    L.ndfl_inflate.argtypes = [vp, vp, u64, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u64), u32]
    L.ndfl_inflate_range.argtypes = [vp, vp, u64, u64, u64, vp, u64, u64, ctypes.POINTER(u64), ctypes.POINTER(u64),
                                     u32]
    L.ndfl_inflate_resolve.argtypes = [vp, ctypes.POINTER(u64)]
    L.ndfl_inflate_tail.argtypes = [vp, u64, vp]
    L.ndfl_inflate_tail_map.argtypes = [vp, u64, vp]
    L.ndfl_inflate_sync.argtypes = [vp, vp, u64, u64, u64, ctypes.POINTER(u64), u32]
    L.ndfl_inflate_headers.argtypes = [vp, vp, u64, u32, ctypes.POINTER(u64), u64, ctypes.POINTER(u64),
                                       ctypes.POINTER(u64), u64, ctypes.POINTER(u64)]
    L.ndfl_bits_shift.argtypes = [vp, vp, u64, u32, vp, u64, u32]
    L.ndfl_crc32.argtypes = [vp, ctypes.POINTER(u32), vp, u64, u32]
    L.ndfl_adler32.argtypes = [vp, ctypes.POINTER(u32), vp, u64, u32]
    L.ndfl_decide.argtypes = [vp, ctypes.POINTER(StrategyNode), u32, u32, vp, u64, u32, u32,
                              ctypes.POINTER(u64), ctypes.POINTER(vp)]
    L.ndfl_compress_to.argtypes = [vp, vp, i32, u32, vp, u64, ctypes.POINTER(u64)]
    L.ndfl_decision_free.argtypes = [vp]
    L.ndfl_crc32_combine.restype = u32
    L.ndfl_crc32_combine.argtypes = [u32, u32, u64]
    _lib = L
    return L


def reason_name(code):
    if code == 0:
        return None
    if 1 <= code <= len(REASONS):
        return REASONS[code - 1]
    return None


class NdflError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = load().ndfl_error_string(code).decode()
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


def check(code, what=""):
    if code < 0:
        raise NdflError(code, what)
    return code
