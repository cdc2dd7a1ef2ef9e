"""GPU parity: libndfl.so's encoder must emit exactly the oracle's bytes (the reference's bytes).

Mirrors T/DeflaterOutputStreamTest.java's cases (empty, short single writes, multi writes, byte
runs, long inputs) but checks bytes against the CPU oracle instead of only round-tripping.
"""
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


def inputs(seed):
    rng = random.Random(seed)
    out = [b"", b"\x00", b"ab", b"aaa", b"\x00" * 1000, b"\x00" * 65536, b"\x00" * 65537, b"\x01" * (1 << 20),
           bytes(range(256)) * 300]
    for n in [1, 2, 3, 63, 64, 65, 100, 1000, 4097, 65535, 65536, 65537, 131072, 200003]:
        out.append(rng.randbytes(n))
        buf = bytearray()
        while len(buf) < n:
            buf += bytes([rng.randrange(3)]) * rng.choice([1, 2, 3, 4, 100, 257, 258, 259, 600, 5000])
        out.append(bytes(buf[:n]))
    return out


@pytest.mark.parametrize("strategy", ["RLE_DYNAMIC", "RLE_STATIC", "LITERAL_DYNAMIC", "LITERAL_STATIC"])
def test_deflate_matches_oracle(ctx, strategy):
    for data in inputs(1):
        got = ctx.deflate(data, strategy)
        exp = O.deflate(data, strategy)
        assert got == exp, (strategy, len(data))


@pytest.mark.parametrize("chunk_len,hist_limit", [(1000, 32768), (64, 1), (777, 0), (65536, 0), (4096, 100)])
def test_deflate_chunk_and_history_params(ctx, chunk_len, hist_limit):
    for data in inputs(2)[::3]:
        for strategy in ["RLE_DYNAMIC", "LITERAL_STATIC"]:
            got = ctx.deflate(data, strategy, chunk_len=chunk_len, hist_limit=hist_limit)
            assert got == O.deflate(data, strategy, chunk_len, hist_limit), (len(data), chunk_len, hist_limit)


def test_crc_fused_into_encoder(ctx):
    for data in inputs(3)[::2]:
        comp, crc = ctx.deflate(data, with_crc=True)
        assert crc == zlib.crc32(data) == O.crc32(data)


def test_crc32_standalone(ctx):
    rng = random.Random(4)
    for n in [0, 1, 7, 64, 65535, 65536, 65537, 1 << 20, 3_000_001]:
        data = rng.randbytes(n)
        assert ctx.crc32(data) == zlib.crc32(data)
        assert ctx.crc32(data, crc=0x12345678) == zlib.crc32(data, 0x12345678)


def test_stream_api_batches_are_bit_exact(ndfl, ctx):
    """DeflaterOutputStream with tiny batches: many GPU calls stitched at odd bit positions must give
    the same bytes as one pass (T/DeflaterOutputStreamTest.java:47-66 style mixed writes)."""
    rng = random.Random(5)
    for _ in range(20):
        data = bytearray()
        while len(data) < 300_000:
            data += bytes([rng.randrange(4)]) * rng.randrange(1, 2000) if rng.random() < 0.5 else rng.randbytes(rng.randrange(1, 3000))
        data = bytes(data[:rng.randrange(0, 300_000)])
        bout = io.BytesIO()
        d = ndfl.DeflaterOutputStream(bout, context=ctx, batch_bytes=rng.choice([1, 65537, 100_000]))
        off = 0
        while off < len(data):
            if rng.random() < 0.1:
                d.write(data[off]); off += 1
            else:
                n = rng.randrange(1, min(70_000, len(data) - off) + 1)
                d.write(data, off, n); off += n
        d.finish()
        assert bout.getvalue() == O.deflate(data)


def test_gzip_config1(ndfl, ctx):
    data = b"\x00" * (1 << 20)
    meta = ndfl.GzipMetadata("DEFLATE", False, 1700000000, 0, "UNIX", None, "zeros_1MiB.bin", None, True)
    bout = io.BytesIO()
    g = ndfl.GzipOutputStream(_NoClose(bout), meta, context=ctx)
    g.write(data)
    g.close()
    exp = O.gzip_compress(data, name=b"zeros_1MiB.bin", mtime=1700000000, os_=3, header_crc=True)
    assert bout.getvalue() == exp


class _NoClose(io.BytesIO):
    def __init__(self, inner):
        super().__init__()
        self.inner = inner

    def write(self, b):
        return self.inner.write(b)

    def close(self):
        pass


def test_large_mixed_corpus_sampled(ctx):
    """64 MiB of the config-4 style corpus: whole output equal to the oracle's."""
    import corpus
    data = corpus.c4_mixed(64 << 20).numpy().tobytes()
    got = ctx.deflate(data)
    exp = O.deflate(data)
    assert len(got) == len(exp) and got == exp
