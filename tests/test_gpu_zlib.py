"""zlib container (D/ZlibMetadata.java, D/ZlibOutputStream.java, D/ZlibInputStream.java) over the
GPU codec, with the GPU Adler-32.  Pinned by Python zlib (adler32, decompress) and the oracle's
container restatement (or_zlib_compress / or_zlib_decompress)."""
import io
import random
import zlib

import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ndfl():
    import ndfl as N
    return N


@pytest.fixture(scope="module")
def ctx(ndfl):
    return ndfl.Context(0)


def datas(seed):
    rng = random.Random(seed)
    out = [b"", b"\x00", b"abc", b"\xff" * 70000, rng.randbytes(65536), rng.randbytes(65537), rng.randbytes(1 << 20)]
    buf = bytearray()
    while len(buf) < 300_000:
        buf += bytes([rng.randrange(4)]) * rng.randrange(1, 700) if rng.random() < 0.5 else rng.randbytes(rng.randrange(1, 500))
    out.append(bytes(buf))
    return out


def test_adler32(ctx):
    rng = random.Random(1)
    for n in [1, 2, 63, 64, 65, 65535, 65536, 65537, 1 << 20, 3_000_017]:
        d = rng.randbytes(n) if n % 2 else b"\xff" * n
        assert ctx.adler32(d) == zlib.adler32(d)
        assert ctx.adler32(d, 0x12345678 % (65521 << 16)) == zlib.adler32(d, 0x12345678 % (65521 << 16))


def test_zlib_output_matches_oracle(ndfl, ctx):
    for data in datas(2):
        bout = io.BytesIO()
        z = ndfl.ZlibOutputStream(_Keep(bout), ndfl.ZlibMetadata.DEFAULT, context=ctx)
        z.write(data)
        z.close()
        got = bout.getvalue()
        assert got == O.zlib_compress(data)
        assert zlib.decompress(got) == data


def test_zlib_input_roundtrip_and_foreign(ndfl, ctx):
    for data in datas(3):
        for comp in [O.zlib_compress(data), zlib.compress(data, 6), zlib.compress(data, 1)]:
            zin = ndfl.ZlibInputStream(io.BytesIO(comp + b"trailing"), context=ctx)
            assert zin.readall() == data
            m = zin.getMetadata()
            assert m.compressionMethod == ndfl.ZlibMetadata.CompressionMethod.DEFLATE


def test_zlib_metadata_roundtrip(ndfl):
    M = ndfl.ZlibMetadata
    for info in range(8):
        for lvl in M.CompressionLevel:
            for dictid in [None, 0xDEADBEEF]:
                m = M(M.CompressionMethod.DEFLATE, info, dictid, lvl)
                hb = m.header_bytes()
                assert ((hb[0] << 8) | hb[1]) % 31 == 0
                assert M.read(io.BytesIO(hb)) == m
    with pytest.raises(ValueError):
        M(M.CompressionMethod.DEFLATE, 8, None, M.CompressionLevel.DEFAULT)


def test_zlib_errors(ndfl, ctx):
    R = ndfl.Reason
    good = O.zlib_compress(b"hello hello hello")

    def reason(stream):
        with pytest.raises(ndfl.DataFormatException) as e:
            ndfl.ZlibInputStream(io.BytesIO(stream), context=ctx).readall()
        return e.value.getReason()

    assert reason(b"") == R.UNEXPECTED_END_OF_STREAM
    assert reason(b"\x78") == R.UNEXPECTED_END_OF_STREAM
    assert reason(bytes([good[0], good[1] ^ 1]) + good[2:]) == R.HEADER_CHECKSUM_MISMATCH
    cmf = 0x77                                             # method 7
    flg = (31 - (cmf << 8) % 31) % 31
    assert reason(bytes([cmf, flg]) + good[2:]) == R.UNSUPPORTED_COMPRESSION_METHOD
    assert reason(good[:-2]) == R.UNEXPECTED_END_OF_STREAM
    bad = bytearray(good); bad[-1] ^= 1
    assert reason(bytes(bad)) == R.DECOMPRESSED_CHECKSUM_MISMATCH
    assert O.zlib_decompress(bytes(bad))[0] == "DECOMPRESSED_CHECKSUM_MISMATCH"
    # compression info 8 with DEFLATE: the record constructor rejects it (IllegalArgumentException)
    cmf = 0x88
    flg = (31 - (cmf << 8) % 31) % 31
    with pytest.raises(ValueError):
        ndfl.ZlibInputStream(io.BytesIO(bytes([cmf, flg]) + good[2:]), context=ctx)


class _Keep(io.BytesIO):
    def __init__(self, inner):
        super().__init__()
        self.inner = inner

    def write(self, b):
        return self.inner.write(b)

    def close(self):
        pass
