"""Gzip container parity on the GPU-backed streams: every gzip Reason of
D/GzipMetadata.java:73-146 and D/GzipInputStream.java:66-90, checked against the oracle's gunzip
(oracle/ndfl_oracle.c, which restates those files), plus headers carrying FEXTRA / FNAME / FCOMMENT /
FTEXT / FHCRC, ISIZE modulo 2^32, trailing bytes after the member and non-seekable (pipe-like) input."""
import io
import zlib

import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

DATA = b"".join(bytes([i % 7]) * (i % 50 + 1) + bytes(range(i % 13)) for i in range(3000))


@pytest.fixture(scope="module")
def ndfl():
    import ndfl as N
    return N


@pytest.fixture(scope="module")
def ctx(ndfl):
    return ndfl.Context(0)


class Pipe(io.RawIOBase):
    """Non-seekable reader that hands out at most `step` bytes per read (a pipe or socket)."""

    def __init__(self, data, step=1000):
        self._d, self._p, self._step = data, 0, step

    def readable(self):
        return True

    def seekable(self):
        return False

    def read(self, n=-1):
        if n is None or n < 0:
            n = len(self._d) - self._p
        n = min(n, self._step)
        b = self._d[self._p:self._p + n]
        self._p += len(b)
        return b


def gpu_gunzip(ndfl, ctx, gz, pipe=False):
    """(reason name or None, output, metadata) through GzipInputStream."""
    src = Pipe(gz) if pipe else io.BytesIO(gz)
    try:
        g = ndfl.GzipInputStream(src, context=ctx)
    except ndfl.DataFormatException as e:
        return e.getReason().name, b"", None
    out = bytearray()
    try:
        while True:
            b = bytearray(7000)
            n = g.read(b, 0, len(b))
            if n == -1:
                break
            out += b[:n]
    except ndfl.DataFormatException as e:
        return e.getReason().name, bytes(out), g.getMetadata()
    return None, bytes(out), g.getMetadata()


def good(**kw):
    return O.gzip_compress(DATA, **kw)


def check(ndfl, ctx, gz, expect):
    oreason, oout, _, _ = O.gunzip(gz)
    greason, gout, meta = gpu_gunzip(ndfl, ctx, gz)
    assert oreason == expect, (oreason, expect)
    assert greason == expect, (greason, expect)
    if expect is None or expect in ("DECOMPRESSED_CHECKSUM_MISMATCH", "DECOMPRESSED_SIZE_MISMATCH"):
        assert gout == oout == DATA
    return meta


def test_header_fields_round_trip(ndfl, ctx):
    gz = good(name=b"file.txt", mtime=1_700_000_000, os_=11, header_crc=True, text=True, comment=b"a comment",
              extra=b"\x01\x02AB\x03\x00xyz", extra_flags=2)
    meta = check(ndfl, ctx, gz, None)
    assert meta.fileName == "file.txt" and meta.comment == "a comment" and meta.isFileText
    assert meta.extraField == b"\x01\x02AB\x03\x00xyz" and meta.extraFlags == 2 and meta.hasHeaderCrc
    assert meta.modificationTimeUnixS == 1_700_000_000 and meta.operatingSystem == "NTFS_FILESYSTEM"
    assert zlib.decompress(gz, 31) == DATA


@pytest.mark.parametrize("os_", [0, 13, 255])
def test_operating_systems_accepted(ndfl, ctx, os_):
    meta = check(ndfl, ctx, good(os_=os_), None)
    assert meta.operatingSystem == ("UNKNOWN" if os_ == 255 else ndfl.streams.OS_NAMES[os_])


def test_invalid_magic(ndfl, ctx):
    gz = bytearray(good())
    gz[1] = 0x8C
    check(ndfl, ctx, bytes(gz), "GZIP_INVALID_MAGIC_NUMBER")


def test_unsupported_method(ndfl, ctx):
    gz = bytearray(good())
    gz[2] = 7
    check(ndfl, ctx, bytes(gz), "UNSUPPORTED_COMPRESSION_METHOD")


@pytest.mark.parametrize("bit", [5, 6, 7])
def test_reserved_flags(ndfl, ctx, bit):
    gz = bytearray(good())
    gz[3] |= 1 << bit
    check(ndfl, ctx, bytes(gz), "GZIP_RESERVED_FLAGS_SET")


@pytest.mark.parametrize("osv", [14, 100, 254])
def test_unsupported_os(ndfl, ctx, osv):
    gz = bytearray(good())
    gz[9] = osv
    check(ndfl, ctx, bytes(gz), "GZIP_UNSUPPORTED_OPERATING_SYSTEM")


def test_header_crc_mismatch(ndfl, ctx):
    gz = bytearray(good(name=b"n", header_crc=True))
    gz[12] ^= 0x40                       # inside the header CRC-16 (after "n\0" at 10..11)
    check(ndfl, ctx, bytes(gz), "HEADER_CHECKSUM_MISMATCH")


def test_decompressed_checksum_mismatch(ndfl, ctx):
    gz = bytearray(good())
    gz[-8] ^= 1
    check(ndfl, ctx, bytes(gz), "DECOMPRESSED_CHECKSUM_MISMATCH")


def test_decompressed_size_mismatch(ndfl, ctx):
    gz = bytearray(good())
    gz[-4] ^= 1
    check(ndfl, ctx, bytes(gz), "DECOMPRESSED_SIZE_MISMATCH")


@pytest.mark.parametrize("cut", [1, 4, 5, 8])
def test_truncated_trailer(ndfl, ctx, cut):
    check(ndfl, ctx, good()[:-cut], "UNEXPECTED_END_OF_STREAM")


@pytest.mark.parametrize("cut", [1, 3, 9, 11])
def test_truncated_header(ndfl, ctx, cut):
    gz = good(name=b"name", comment=b"c", extra=b"\x00\x01", header_crc=True)
    hdr_len = 10 + 2 + 2 + 5 + 2 + 2
    check(ndfl, ctx, gz[:hdr_len - cut], "UNEXPECTED_END_OF_STREAM")


def test_trailing_bytes_ignored(ndfl, ctx):
    check(ndfl, ctx, good() + b"\x1f\x8bgarbage", None)


def test_isize_modulo_2_32(ndfl, ctx):
    """ISIZE is the length mod 2^32 (D/GzipOutputStream.java:69, D/GzipInputStream.java:87): 4 GiB +
    12,345 zero bytes written through GzipOutputStream in 256 MiB pieces carry ISIZE 12,345, and
    GzipInputStream accepts the member."""
    n = (1 << 32) + 12345
    piece = bytes(256 << 20)
    b = io.BytesIO()
    meta = ndfl.GzipMetadata("DEFLATE", False, None, 0, "UNIX", None, None, None, False)
    g = ndfl.GzipOutputStream(b, meta, context=ctx)
    left = n
    while left:
        k = min(left, len(piece))
        g.write(piece, 0, k)
        left -= k
    g.finish()
    gz = b.getvalue()
    assert int.from_bytes(gz[-4:], "little") == 12345
    crc = 0
    for _ in range(16):
        crc = zlib.crc32(piece, crc)
    assert int.from_bytes(gz[-8:-4], "little") == zlib.crc32(bytes(12345), crc)
    r = ndfl.GzipInputStream(io.BytesIO(gz), context=ctx)
    total = 0
    buf = bytearray(1 << 28)
    while (k := r.read(buf, 0, len(buf))) != -1:
        assert buf[:k].count(0) == k
        total += k
    assert total == n


def test_non_seekable_input(ndfl, ctx):
    gz = good(name=b"p", header_crc=True)
    r, out, meta = gpu_gunzip(ndfl, ctx, gz, pipe=True)
    assert r is None and out == DATA and meta.fileName == "p"


def test_zlib_non_seekable_input(ndfl, ctx):
    z = O.zlib_compress(DATA)
    zi = ndfl.ZlibInputStream(Pipe(z), context=ctx)
    assert zi.readall() == DATA
