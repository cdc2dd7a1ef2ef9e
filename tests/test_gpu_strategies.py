"""GPU parity of the position-dependent strategies: Uncompressed (D/comp/Uncompressed.java) and
MultiStrategy (D/comp/MultiStrategy.java), against the oracle (itself N-version-pinned to
tests/pyref_deflate.py in tests/test_oracle_deflate.py)."""
import io
import random
import zlib

import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

PR = {"LITERAL_STATIC": (False, 0, 0, 0, 0), "LITERAL_DYNAMIC": (True, 0, 0, 0, 0),
      "RLE_STATIC": (False, 3, 258, 1, 1), "RLE_DYNAMIC": (True, 3, 258, 1, 1),
      "FULL_STATIC": (False, 3, 258, 1, 32768), "FULL_DYNAMIC": (True, 3, 258, 1, 32768)}


@pytest.fixture(scope="module")
def ndfl():
    import ndfl as N
    return N


@pytest.fixture(scope="module")
def ctx(ndfl):
    return ndfl.Context(0)


def inputs(seed):
    rng = random.Random(seed)
    out = [b"", b"\x00", b"ab", b"\x00" * 65535, b"\x00" * 65536, b"\x00" * 65537, b"\x00" * 131071,
           bytes(range(256)) * 700]
    for n in [1, 5, 64, 1000, 65535, 65536, 65537, 200003]:
        out.append(rng.randbytes(n))
        buf = bytearray()
        while len(buf) < n:
            buf += bytes([rng.randrange(3)]) * rng.choice([1, 2, 100, 258, 600]) if rng.random() < 0.5 \
                else rng.randbytes(rng.randrange(1, 300))
        out.append(bytes(buf[:n]))
    return out


def _subs(ndfl, names):
    return [ndfl.Uncompressed.SINGLETON if n == "UNCOMPRESSED" else ndfl.Lz77Huffman(*PR[n]) for n in names]


def _osubs(names):
    return ["UNCOMPRESSED" if n == "UNCOMPRESSED" else PR[n] for n in names]


def test_uncompressed_matches_oracle(ctx):
    for data in inputs(21):
        for chunk_len in [65536, 1000, 65535, 70]:
            got = ctx.deflate(data, "UNCOMPRESSED", chunk_len=chunk_len)
            assert got == O.deflate(data, "UNCOMPRESSED", chunk_len), (len(data), chunk_len)
            assert zlib.decompress(got, -15) == data


@pytest.mark.parametrize("names", [["RLE_DYNAMIC", "UNCOMPRESSED"], ["UNCOMPRESSED", "LITERAL_STATIC"],
                                   ["LITERAL_DYNAMIC", "RLE_STATIC", "UNCOMPRESSED", "FULL_DYNAMIC"],
                                   ["FULL_STATIC", "FULL_DYNAMIC", "RLE_DYNAMIC"], ["RLE_DYNAMIC"]])
def test_multistrategy_matches_oracle(ndfl, ctx, names):
    strat = ndfl.MultiStrategy(*_subs(ndfl, names))
    for data in inputs(22)[::2]:
        for chunk_len, hist in [(65536, 32768), (999, 32768), (4096, 0)]:
            got = ctx.deflate(data, strat, chunk_len=chunk_len, hist_limit=hist)
            exp = O.deflate_multi(data, _osubs(names), chunk_len, hist)
            assert got == exp, (names, len(data), chunk_len, hist)
            reason, out, _ = ctx.inflate(got)
            assert reason is None and out == data


def test_multistrategy_stream_batches(ndfl, ctx):
    """Odd start bit positions across GPU calls change the Uncompressed lengths and thus the choice."""
    rng = random.Random(23)
    strat = ndfl.MultiStrategy(ndfl.Lz77Huffman.RLE_DYNAMIC, ndfl.Uncompressed.SINGLETON)
    for _ in range(6):
        data = b"".join(inputs(rng.randrange(100))[rng.randrange(8, 24)] for _ in range(3))
        bout = io.BytesIO()
        d = ndfl.DeflaterOutputStream(bout, dataLookaheadLimit=rng.choice([65536, 5000]), strategy=strat,
                                      context=ctx, batch_bytes=rng.choice([1, 65537, 100_000]))
        off = 0
        while off < len(data):
            n = rng.randrange(1, min(90_000, len(data) - off) + 1)
            d.write(data, off, n)
            off += n
        d.finish()
        assert bout.getvalue() == O.deflate_multi(data, _osubs(["RLE_DYNAMIC", "UNCOMPRESSED"]), d._chunk)


def test_multistrategy_validation(ndfl):
    with pytest.raises(ValueError):
        ndfl.MultiStrategy()
    with pytest.raises(TypeError):
        ndfl.MultiStrategy(None)


@pytest.mark.parametrize("name,m", [("RLE_DYNAMIC", 1024), ("FULL_DYNAMIC", 4096), ("LITERAL_STATIC", 64),
                                    ("RLE_STATIC", 30000)])
def test_binarysplit_matches_oracle(ndfl, ctx, name, m):
    strat = ndfl.BinarySplit(ndfl.Lz77Huffman(*PR[name]), m)
    for data in inputs(24)[::2] + [inputs(25)[-1] * 3]:
        for chunk_len, hist in [(65536, 32768), (65536, 0), (8192, 100)]:
            got = ctx.deflate(data, strat, chunk_len=chunk_len, hist_limit=hist)
            exp = O.deflate_binsplit(data, PR[name], m, chunk_len, hist)
            assert got == exp, (name, m, len(data), chunk_len, hist)
            reason, out, _ = ctx.inflate(got)
            assert reason is None and out == data


def test_binarysplit_stream_batches(ndfl, ctx):
    rng = random.Random(26)
    strat = ndfl.BinarySplit(ndfl.Lz77Huffman.RLE_DYNAMIC, 2048)
    for _ in range(4):
        data = b"".join(inputs(rng.randrange(100))[rng.randrange(8, 24)] for _ in range(3))
        bout = io.BytesIO()
        d = ndfl.DeflaterOutputStream(bout, strategy=strat, context=ctx, batch_bytes=rng.choice([1, 65537, 300_000]))
        off = 0
        while off < len(data):
            n = rng.randrange(1, min(90_000, len(data) - off) + 1)
            d.write(data, off, n)
            off += n
        d.finish()
        assert bout.getvalue() == O.deflate_binsplit(data, PR["RLE_DYNAMIC"], 2048)


def test_binarysplit_validation(ndfl):
    with pytest.raises(ValueError):
        ndfl.BinarySplit(ndfl.Lz77Huffman.RLE_DYNAMIC, 0)
    with pytest.raises(TypeError):
        ndfl.BinarySplit(None, 5)
