"""CPU-side checks of the drop-in boundary: libndfl.so builds for gfx950, loads, and exports every
symbol include/ndfl.h declares.  No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deflate-library-java_amd")


def _lib_path():
    path = os.path.join(PKG, "lib", "libndfl.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", PKG])
    return path


def test_header_symbols_exported():
    hdr = open(os.path.join(ROOT, "include", "ndfl.h")).read()
    declared = set(re.findall(r"^\s*(?:int|uint32_t|uint64_t|double|const char\*)\s+(ndfl_\w+)\(", hdr, re.M))
    assert len(declared) >= 10
    lib = ctypes.CDLL(_lib_path())
    for name in sorted(declared):
        assert hasattr(lib, name), name
    import ndfl._lib as L
    assert set(L.EXPORTS) == declared


def test_abi_version_and_error_strings():
    lib = ctypes.CDLL(_lib_path())
    lib.ndfl_abi_version.restype = ctypes.c_uint32
    assert lib.ndfl_abi_version() == 1
    lib.ndfl_error_string.restype = ctypes.c_char_p
    assert lib.ndfl_error_string(1) == b"Unexpected end of stream"
    assert lib.ndfl_error_string(12) == b"Attempting to copy from before start of dictionary"


def test_ctx_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        return
    lib = ctypes.CDLL(_lib_path())
    h = ctypes.c_void_p()
    assert lib.ndfl_ctx_create(ctypes.byref(h), 0, 0) == -4     # NDFL_E_DEVICE, no silent fallback


def test_crc32_combine_host():
    import zlib
    lib = ctypes.CDLL(_lib_path())
    lib.ndfl_crc32_combine.restype = ctypes.c_uint32
    lib.ndfl_crc32_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
    a, b = b"hello ", b"world" * 1000
    assert lib.ndfl_crc32_combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(a + b)


def test_header_constants_match_python_binding():
    """The flag / size constants of include/ndfl.h and the ctypes binding agree (the kernels
    static_assert the pad size against the header themselves)."""
    hdr = open(os.path.join(ROOT, "include", "ndfl.h")).read()
    consts = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define NDFL_(\w+)\s+\(?(-?\d+)u?\)?", hdr)}
    import ndfl._lib as L
    assert consts["IN_DEVICE"] == L.IN_DEVICE and consts["OUT_DEVICE"] == L.OUT_DEVICE
    assert consts["DICT_DEFERRED"] == L.DICT_DEFERRED and consts["IN_PADDED"] == L.IN_PADDED
    assert consts["IN_PAD_BYTES"] == L.IN_PAD_BYTES and consts["IN_PARTIAL"] == L.IN_PARTIAL
    assert consts["NEED_INPUT"] == L.NEED_INPUT and consts["E_CAPACITY"] == L.E_CAPACITY
